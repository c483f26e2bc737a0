#!/bin/bash
# Flat nq=1 merge latency + IVF per-step kernel trace (nq 1024 and 1)
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/flat_latency.py > gpurun_out/r03_flat_latency.log 2>&1 || { tail -20 gpurun_out/r03_flat_latency.log; exit 1; }
tail -2 gpurun_out/r03_flat_latency.log
cd /tmp && export TMPDIR=/tmp
for nq in 1024 1; do
  rm -rf "$root/gpurun_out/trace_ivf_nq$nq"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivf_nq$nq" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq $nq --steps 20 --warmup 3 \
      > "$root/gpurun_out/trace_ivf_nq$nq.log" 2>&1 || exit 1
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_ivf_nq$nq" | head -30
done
