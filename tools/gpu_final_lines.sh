#!/usr/bin/env bash
# The round's bench lines: default (IVF, with CPU baseline), Flat 1M and 10M (L2, IP), DiskANN C4.
#   tools/gpu_final_lines.sh → gpurun_out/final_*.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
run() {  # name, args...
    local name="$1"; shift
    timeout -k 10 400 python -u bench.py "$@" > "gpurun_out/final_$name.json" 2> "gpurun_out/final_$name.err" || exit 1
    echo "$name $(grep -o '"value": [0-9.]*\|"recall_at_10": [0-9.]*\|"frac": [0-9.]*' "gpurun_out/final_$name.json" | tr '\n' ' ')"
}
run ivf10m
run flat1m --workload flat --n 1000000 --no-cpu-baseline
run flat10m_ip --workload flat --metric ip --no-cpu-baseline
run diskann1m --workload diskann
