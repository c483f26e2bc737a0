#!/bin/bash
# r05: timing ablations of the Flat int8 bounded-pass kernel at 10M x 768 (tuning builds in abl/, wrong results:
# only kernel_ms is read).  bit 0 no tile DMA, 1 no query-fragment loads, 2 no epilogue filter, 3 no barrier,
# 4 no append path.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', r.get('kernel_ms'), r.get('frac'))"; }
timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | line "full" || exit 1
for lib in abl/*.so; do
  HIPANN_LIB=$lib timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | line "$lib" || exit 1
done
