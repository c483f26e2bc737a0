#!/usr/bin/env bash
# SQ counters + FETCH_SIZE of the bench's IVF scan, each set in its own pass (no trace domains beside
# --pmc).  HIPANN_LIB selects a tuning build.  → gpurun_out/pmc_<tag>_{sq,fetch}/
#   tools/pmc_sq.sh <tag> [extra bench args...]
set -euo pipefail
tag="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-include-regex ivf_scan --output-format csv -d "$root/gpurun_out/pmc_${tag}_sq" -o run -- python3 "$root/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" \
    > "$root/gpurun_out/pmc_${tag}_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
    --kernel-include-regex ivf_scan --output-format csv -d "$root/gpurun_out/pmc_${tag}_fetch" -o run -- python3 "$root/bench.py" --no-cpu-baseline --steps 2 --warmup 1 "$@" \
    > "$root/gpurun_out/pmc_${tag}_fetch.log" 2>&1
