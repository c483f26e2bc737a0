#!/bin/bash
# r03: IVF per-batch cost outside the scan — GPU tests of the IVF / Flat paths, then kernel traces of the
# 1024-query step (default, and HIPANN_KEYS=0: the one-pass coarse key kernel) summarised per step.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ivf_gpu.py tests/test_flat_gpu.py tests/test_configs_gpu.py > gpurun_out/ivfcost_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/ivfcost_tests.log; exit 1; }
tail -1 gpurun_out/ivfcost_tests.log
fi
cd /tmp && export TMPDIR=/tmp
root="$GRAFT_REPO_ROOT"
for v in default 0; do
  if [ $v = default ]; then unset HIPANN_KEYS; else export HIPANN_KEYS=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivfc_$v" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq 1024 --steps 30 --warmup 3 \
      > "$root/gpurun_out/trace_ivfc_$v.log" 2>&1 || { echo "trace failed"; tail -5 "$root/gpurun_out/trace_ivfc_$v.log"; exit 1; }
  grep -o '"value": [0-9.]*, "unit": "queries/s", "n_gpus": 1, "steps": 30, "warmup": 3, "ms_per_step": [0-9.]*' "$root/gpurun_out/trace_ivfc_$v.log"
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_ivfc_$v" ivf_scan_mfma_h 8 > "$root/gpurun_out/ivfc_breakdown_$v.txt"
  cat "$root/gpurun_out/ivfc_breakdown_$v.txt"
done
