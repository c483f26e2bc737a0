#!/bin/bash
# r05: fused int8 query preparation (HIPANN_I8_PREP_FUSED) A/B on C2 and Flat 10M (same box, alternating), then the
# Flat parity tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', l['value'], l['ms_per_step'], r.get('kernel_ms'), r.get('frac'))"; }
for ab in HIPANN_I8_PREP_FUSED=0 HIPANN_I8_PREP_FUSED=1 HIPANN_I8_PREP_FUSED=0 HIPANN_I8_PREP_FUSED=1; do
  export "$ab"
  timeout -k 10 300 python -u bench.py --workload flat --n 1000000 --no-alt-forms --no-cpu-baseline --steps 40 --warmup 5 2>/dev/null | line "$ab C2" || exit 1
done
export HIPANN_I8_PREP_FUSED=1
timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | line "fused 10M" || exit 1
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py tests/test_flat_kth_gpu.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flat or c2 or bounded or c5" > gpurun_out/r05_prep_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_prep_tests.log; exit $rc
