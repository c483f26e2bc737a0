#!/usr/bin/env bash
# Kernel traces of the IVF path: the 1024-query batch and the extension's nq = 1 call
#   → gpurun_out/trace_ivf_nq{1024,1}/ (rocprofv3 csv)
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for nq in 1024 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivf_nq$nq" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq $nq --steps 10 --warmup 3 \
      > "$root/gpurun_out/trace_ivf_nq$nq.log" 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$root/gpurun_out/trace_ivf_nq$nq.log"
done
