#!/usr/bin/env bash
# Kernel trace of the default IVF bench (no alt forms) → gpurun_out/trace_ivf/
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivf" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms > "$root/gpurun_out/trace_ivf.log" 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' "$root/gpurun_out/trace_ivf.log"
