#!/bin/bash
# r06: kernel trace of the C4 host-BFS path (the id-gather launches per lock-step step) — per-kernel stats.
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/r06bfs_trace" -o run -- \
    python3 "$root/bench.py" --workload diskann --n 1000000 --d 1536 --diskann-host-bfs --no-cpu-baseline --no-suite \
    --steps 3 --warmup 1 > "$root/gpurun_out/r06bfs_trace.log" 2>&1 || { tail -5 "$root/gpurun_out/r06bfs_trace.log"; exit 1; }
head -8 "$root/gpurun_out/r06bfs_trace/run_kernel_stats.csv" | cut -c1-250
