#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flat_gpu.py tests/test_configs_gpu.py -k "flat or c1" > gpurun_out/r03_flat_tests.log 2>&1 || { tail -40 gpurun_out/r03_flat_tests.log; exit 1; }
tail -2 gpurun_out/r03_flat_tests.log
timeout -k 10 300 python -u tools/flat_latency.py 2>&1 | tee gpurun_out/r03_flat_latency.log
