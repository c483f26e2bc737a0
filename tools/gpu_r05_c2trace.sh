#!/bin/bash
# r05: C2 (Flat L2 1M x 768, nq 1024) per-step kernel breakdown from a rocprofv3 kernel trace (anchor: the keys-mode
# seed pass, one per step).
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/c2tr" -o run -- \
    python3 "$root/bench.py" --workload flat --n 1000000 --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 5 \
    > "$root/gpurun_out/c2tr.log" 2>&1 ) || { tail -5 gpurun_out/c2tr.log; exit 1; }
python3 tools/trace_summary.py gpurun_out/c2tr "flat_bf16_k64<true, true" 5
