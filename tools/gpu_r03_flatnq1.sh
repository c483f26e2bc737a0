#!/bin/bash
# r03: kernel trace of Flat 10M x 768 at nq = 1 / 4 (the extension's per-query call): scan + two-level merge.
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/trace_flat_nq1" -o run -- \
    python3 "$root/tools/flat_latency.py" > "$root/gpurun_out/trace_flat_nq1.log" 2>&1 || { tail -5 "$root/gpurun_out/trace_flat_nq1.log"; exit 1; }
grep -E "nq=|ms_per_call" "$root/gpurun_out/trace_flat_nq1.log" | cut -c1-400
