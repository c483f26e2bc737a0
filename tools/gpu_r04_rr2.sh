#!/bin/bash
# r04: rerank with the single-barrier wave select — the IVF / Flat exact-form tests, the rerank phase clocks, the
# per-step trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ivf_gpu.py tests/test_request_k_gpu.py tests/test_configs_gpu.py tests/test_flat_gpu.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_rr2_tests.log 2>&1 \
    || { echo "tests failed"; tail -60 gpurun_out/r04_rr2_tests.log; exit 1; }
tail -1 gpurun_out/r04_rr2_tests.log
bash tools/gpu_r04_rrprof.sh && bash tools/gpu_r04_ivfcost.sh
