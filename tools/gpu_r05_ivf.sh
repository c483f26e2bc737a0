#!/bin/bash
# r05: IVF headline step A/B (IVF_AB="VAR=a VAR=b", same box) with a kernel-trace breakdown per setting, then the
# IVF parity tests.  Stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', l['value'], l['ms_per_step'], r.get('kernel_ms'), r.get('frac'), l.get('ids_eq_cpu_path'))"; }
for ab in ${IVF_AB:-DEFAULT=1}; do
  export "$ab"
  timeout -k 10 300 python -u bench.py --no-alt-forms --no-cpu-baseline --no-suite --no-c5 --steps 20 --warmup 5 2>/dev/null | line "$ab" || exit 1
  tag=$(echo "$ab" | tr '=/' '__')
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/ivftr_$tag" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 5 > "$root/gpurun_out/ivftr_$tag.log" 2>&1 ) || exit 1
  python3 tools/trace_summary.py "gpurun_out/ivftr_$tag" ivf_scan_mfma_h 5 || exit 1
done
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 700 python -u -m pytest tests/test_ivf_gpu.py tests/test_configs_gpu.py tests/test_distributed.py tests/test_request_k_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ivf or c3 or coarse or partitioned" > gpurun_out/r05_ivf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_ivf_tests.log; exit $rc
