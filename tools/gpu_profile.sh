#!/usr/bin/env bash
# Profile one bench workload on the GPU box: a kernel-trace/stats pass and a separate FETCH_SIZE
# PMC pass (MI355X_MICROARCH.md §HBM: counters in their own run, no trace domains beside --pmc).
#   tools/gpu_profile.sh <workload> <kernel-substring> <key> [extra bench args...]
# <key> names the configuration the traffic belongs to (bench.py pmc_traffic: e.g. ivf_10000000x768,
# flat_1000000x768, diskann_1000000x1536).
# Outputs: gpurun_out/prof_<key>/{stats,pmc}/..., gpurun_out/pmc_<key>.json
set -euo pipefail
wl="$1"; kern="$2"; key="$3"; shift 3
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/prof_$key"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
    python3 "$root/bench.py" --workload "$wl" --no-cpu-baseline --no-suite "$@" > "$out/stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$kern" --output-format csv -d "$out/pmc" -o run -- \
    python3 "$root/bench.py" --workload "$wl" --no-cpu-baseline --no-suite "$@" > "$out/pmc.log" 2>&1
python3 "$root/tools/pmc_traffic.py" "$out/pmc" "$kern" --skip 3 --per-step "${PER_STEP:-1}" --out "$root/gpurun_out/pmc_$key.json"
