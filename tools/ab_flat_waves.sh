#!/usr/bin/env bash
# A/B of the split Flat kernel's block shape: 4-wave (128-query) vs 8-wave (256-query) blocks.
#   tools/ab_flat_waves.sh   → gpurun_out/ab_flat_w{4,8}.json, gpurun_out/pytest_flat_w8.log
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
HIPANN_FLAT_BF_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_flat_w8.log 2>&1 || { tail -30 gpurun_out/pytest_flat_w8.log; exit 1; }
tail -1 gpurun_out/pytest_flat_w8.log
for w in 4 8; do
    HIPANN_FLAT_BF_WAVES=$w timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --steps 3 --warmup 1 \
        > gpurun_out/ab_flat_w$w.json 2> gpurun_out/ab_flat_w$w.err || exit 1
    echo "w=$w $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/ab_flat_w$w.json | tr '\n' ' ')"
done
