#!/bin/bash
# r03: new/changed GPU tests first, then the whole -m gpu suite, smoke and the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_configs_gpu.py tests/test_harness_gpu.py tests/test_distributed.py \
  -k "rccl or c1_ or duplicate or harness or flow" > gpurun_out/r03_new.log 2>&1 || { echo "new tests failed"; tail -50 gpurun_out/r03_new.log; exit 1; }
timeout -k 10 600 $T tests/test_ivf_gpu.py -k "ties or fallback" > gpurun_out/r03_ties.log 2>&1 || { echo "tie tests failed"; tail -60 gpurun_out/r03_ties.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_suite.log 2>&1 || { echo "suite failed"; tail -60 gpurun_out/r03_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03_bench.err; exit 1; }
echo bench ok
