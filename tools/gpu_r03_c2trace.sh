#!/bin/bash
# C2 (Flat 1M x 768 L2, nq 1024) and Flat 10M per-step kernel breakdown (rocprofv3 kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for n in 1000000 10000000; do
  rm -rf "$root/gpurun_out/trace_flat_$n"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_flat_$n" -o run -- \
      python3 "$root/bench.py" --workload flat --n $n --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 \
      --warmup 3 > "$root/gpurun_out/trace_flat_$n.log" 2>&1 || exit 1
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_flat_$n" flat_keys_kth 5 | head -20
done
