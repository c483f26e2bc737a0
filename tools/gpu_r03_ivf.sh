#!/bin/bash
# IVF changes: IVF + config + distributed GPU tests, then the per-step kernel trace at nq 1024 and 1
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ivf_gpu.py tests/test_configs_gpu.py tests/test_distributed.py tests/test_harness_gpu.py -m gpu > gpurun_out/r03_ivf_tests.log 2>&1 || { tail -60 gpurun_out/r03_ivf_tests.log; exit 1; }
tail -2 gpurun_out/r03_ivf_tests.log
cd /tmp && export TMPDIR=/tmp
for nq in 1024 1; do
  rm -rf "$root/gpurun_out/trace_ivf_nq$nq"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivf_nq$nq" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq $nq --steps 20 --warmup 3 \
      > "$root/gpurun_out/trace_ivf_nq$nq.log" 2>&1 || exit 1
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_ivf_nq$nq" | head -30
done
