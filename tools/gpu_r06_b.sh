#!/bin/bash
# r06b: the C3 / IVF GPU tests with failure details, then the σ = 0.3 mixture probe (per form: time, flagged queries).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_ivf_gpu.py -m gpu -q -rf --maxfail=20 \
    --timeout 300 --timeout-method thread > gpurun_out/r06b_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r06b_tests.log | cut -c1-600
cat gpurun_out/probe_parity.json 2>/dev/null | head -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc"; exit 1; fi
timeout -k 10 400 python -u tools/ivf_clustered_probe.py 0.3 10000000 1,8 6,5,3 > gpurun_out/r06b_probe.log 2>&1 || { tail -20 gpurun_out/r06b_probe.log; exit 1; }
cat gpurun_out/r06b_probe.log
