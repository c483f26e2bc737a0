#!/bin/bash
# r05: Flat int8 kernel timing at 10M x 768 and C2 (1M x 768), then the Flat parity tests.  Stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', l['value'], l['ms_per_step'], r.get('kernel_ms'), r.get('merge_ms'), r.get('frac'))"; }
# FLAT_AB="VAR=a VAR=b": each setting's timing lines (same box), else the default build's
for ab in ${FLAT_AB:-DEFAULT=1}; do
export "$ab"
timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | line "$ab 10M" || exit 1
timeout -k 10 300 python -u bench.py --workload flat --n 1000000 --no-alt-forms --no-cpu-baseline --steps 20 --warmup 3 2>/dev/null | line "$ab C2" || exit 1
timeout -k 10 300 python -u bench.py --workload flat --n 12500000 --metric ip --no-alt-forms --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | line "$ab C5ip" || exit 1
done
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 700 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py tests/test_flat_kth_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "flat or c2 or bounded or c5" > gpurun_out/r05_flat_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_flat_tests.log; exit $rc
