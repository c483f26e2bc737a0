#!/bin/bash
# r03 end-of-round evidence on the final tree: the whole -m gpu suite, smoke, the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_suite.log 2>&1 || { echo "suite failed"; tail -60 gpurun_out/r03_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r03_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03_bench.err; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r03_bench.json | head -1
