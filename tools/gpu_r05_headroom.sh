#!/bin/bash
# r05: device-buffer regrowth headroom (HIPANN_BUF_HEADROOM) A/B on the append + search line (same box), then the
# IVF / Flat parity tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for ab in HIPANN_BUF_HEADROOM=0 HIPANN_BUF_HEADROOM=1; do
  export "$ab"
  timeout -k 10 400 python -u bench.py --no-alt-forms --no-cpu-baseline --no-c5 --steps 10 --warmup 3 > gpurun_out/hr.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.loads(open('gpurun_out/hr.json').read().strip().splitlines()[-1]); print('$ab', l['ms_per_step'], l['append2048'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_hr_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05_hr_tests.log; exit $rc
