#!/usr/bin/env bash
# Flat parity tests (tools/gpu_flat_check.sh: Flat + IVF tests, the L2 bench line with the other forms),
# then the 10M x 768 IP bench line.
#   tools/gpu_flat_lines.sh → gpurun_out/pytest_flat.log, gpurun_out/bench_flat.json, gpurun_out/final_flat10m_ip.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
bash tools/gpu_flat_check.sh > gpurun_out/fc.log 2>&1 || { tail -c 2000 gpurun_out/fc.log; exit 1; }
tail -c 600 gpurun_out/fc.log
timeout -k 10 300 python -u bench.py --workload flat --metric ip --no-cpu-baseline --no-alt-forms \
    > gpurun_out/final_flat10m_ip.json 2> gpurun_out/final_flat10m_ip.err || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"merge_ms": [0-9.]*\|"frac": [0-9.]*\|rerank_fallbacks_total.: [0-9]*\|"ms_per_step": [0-9.]*' \
    gpurun_out/final_flat10m_ip.json
