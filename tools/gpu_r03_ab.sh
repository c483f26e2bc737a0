#!/bin/bash
# IVF fixed-cost A/B: per-step kernel traces (nq 1024) under environment variants given as arguments,
# e.g. tools/gpu_r03_ab.sh "" "HIPANN_KEYS=0" "HIPANN_ROWSEL_WAVE=1"
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  rm -rf "$root/gpurun_out/trace_ab$i"
  echo "== variant $i: [$v]"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ab$i" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 3 \
      > "$root/gpurun_out/trace_ab$i.log" 2>&1 || exit 1
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_ab$i" | head -14
done
