#!/usr/bin/env bash
# Flat (+ IVF, whose coarse quantizer is a Flat index) parity tests, then the Flat bench line with the
# other q·x forms timed beside it — one GPU call.
#   tools/gpu_flat_check.sh   → gpurun_out/pytest_flat.log, gpurun_out/bench_flat.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_flat_gpu.py tests/test_ivf_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_flat.log 2>&1 || { tail -40 gpurun_out/pytest_flat.log; exit 1; }
tail -1 gpurun_out/pytest_flat.log
timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --steps 3 --warmup 1 \
    > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.err
rc=$?
tail -c 3000 gpurun_out/bench_flat.json
exit $rc
