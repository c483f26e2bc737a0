#!/bin/bash
# r04: Flat form 5 (int8 filter) — targeted parity tests, then the 10M x 768 Flat line at forms 5 and 4, then C5's
# shard (12.5M IP).  Each step under its own time limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py tests/test_request_k_gpu.py tests/test_configs_gpu.py -x -q \
    --timeout 300 --timeout-method thread -k "i8 or two_pass or candidate_rerank or forms_blas or bounded_passes or c2_flat or large_batch" \
    > gpurun_out/r04_i8_tests.log 2>&1 || { echo "i8 tests failed"; tail -60 gpurun_out/r04_i8_tests.log; exit 1; }
tail -1 gpurun_out/r04_i8_tests.log
timeout -k 10 600 python -u -m pytest tests/test_ivf_gpu.py tests/test_request_k_gpu.py tests/test_configs_gpu.py -x -q \
    --timeout 300 --timeout-method thread -k "fallback or ties or half_form or exact_form or ivf_exact_forms_request_k or c3" \
    > gpurun_out/r04_ivf_fb_tests.log 2>&1 || { echo "ivf fallback tests failed"; tail -60 gpurun_out/r04_ivf_fb_tests.log; exit 1; }
tail -1 gpurun_out/r04_ivf_fb_tests.log
timeout -k 10 300 python -u -m pytest tests/test_harness_gpu.py tests/test_ivf_train_gpu.py -x -q --timeout 240 \
    --timeout-method thread > gpurun_out/r04_harness.log 2>&1 || { echo "harness failed"; tail -40 gpurun_out/r04_harness.log; \
    grep FAIL gpurun_out/faiss_index_harness.log | head; exit 1; }
tail -1 gpurun_out/r04_harness.log
for f in 5 4; do
  HIPANN_FLAT_FORM=$f timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --steps 10 --warmup 2 \
      > gpurun_out/r04_flat10m_f$f.json 2> gpurun_out/r04_flat10m_f$f.err || { echo "flat form $f failed"; tail -20 gpurun_out/r04_flat10m_f$f.err; exit 1; }
  cat gpurun_out/r04_flat10m_f$f.json
done
HIPANN_FLAT_FORM=5 timeout -k 10 300 python -u bench.py --workload flat --metric ip --n 12500000 --no-cpu-baseline \
    --steps 10 --warmup 2 > gpurun_out/r04_c5_f5.json 2> gpurun_out/r04_c5_f5.err || { echo "c5 form 5 failed"; tail -20 gpurun_out/r04_c5_f5.err; exit 1; }
cat gpurun_out/r04_c5_f5.json
