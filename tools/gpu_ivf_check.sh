#!/usr/bin/env bash
# IVF parity tests, then the default IVF bench line — one GPU call.
#   tools/gpu_ivf_check.sh [extra bench args...]   → gpurun_out/pytest_ivf.log, gpurun_out/bench_ivf.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ivf_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_ivf.log 2>&1 || { tail -30 gpurun_out/pytest_ivf.log; exit 1; }
tail -1 gpurun_out/pytest_ivf.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_ivf.json 2> gpurun_out/bench_ivf.err
rc=$?
tail -c 3000 gpurun_out/bench_ivf.json
exit $rc
