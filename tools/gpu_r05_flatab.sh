#!/bin/bash
# r05: Flat int8 kernel A/B (HIPANN_FLAT_W4: the 4-wave, 512-register variant) at 10M x 768 and C2, plus
# correctness of the variant on the Flat int8 parity tests.  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', l['value'], l['ms_per_step'], r.get('kernel_ms'), r.get('merge_ms'), r.get('frac'))"; }
for w in 0 1; do
  HIPANN_FLAT_W4=$w timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | line "w4=$w 10M" || exit 1
  HIPANN_FLAT_W4=$w timeout -k 10 300 python -u bench.py --workload flat --n 1000000 --no-alt-forms --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | line "w4=$w C2" || exit 1
done
HIPANN_FLAT_W4=1 timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "i8 or c2 or bounded or successive or multi_shard or nan" > gpurun_out/r05_w4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_w4_tests.log; exit $rc
