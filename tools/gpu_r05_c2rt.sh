#!/bin/bash
# r05: C2 (Flat L2 1M x 768, nq 1024) HIP runtime-API + kernel trace (no counters), for the host-side time per step.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d "$root/gpurun_out/c2rt" -o run -- \
    python3 "$root/bench.py" --workload flat --n 1000000 --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 5 \
    > "$root/gpurun_out/c2rt.log" 2>&1 ) || { tail -5 gpurun_out/c2rt.log; exit 1; }
ls gpurun_out/c2rt/*/ 2>/dev/null | head; ls gpurun_out/c2rt
