#!/bin/bash
# r04: Flat nq < 20 on the int8 image (flat_i8_scan) — the small-batch tests, then the 10M x 768 latency at nq 1/4/16
# against the fp32 direct scan (HIPANN_FLAT_I8_SMALL=0).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py -x -q --timeout 300 --timeout-method thread -k "small_batch or batch_sizes or k_range or odd_dim or sql_known or faiss_metal or large_prop or ties" \
    > gpurun_out/r04_i8small_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r04_i8small_tests.log; exit 1; }
tail -1 gpurun_out/r04_i8small_tests.log
timeout -k 10 300 python -u tools/flat_latency.py > gpurun_out/r04_flat_latency_i8.txt 2>&1 || { tail -20 gpurun_out/r04_flat_latency_i8.txt; exit 1; }
cat gpurun_out/r04_flat_latency_i8.txt
HIPANN_FLAT_I8_SMALL=0 timeout -k 10 300 python -u tools/flat_latency.py > gpurun_out/r04_flat_latency_fp32.txt 2>&1 || { tail -20 gpurun_out/r04_flat_latency_fp32.txt; exit 1; }
cat gpurun_out/r04_flat_latency_fp32.txt
