#!/usr/bin/env bash
# IVF parity tests + the default IVF bench line without the alt forms (quick A/B of the per-batch path).
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ivf_gpu.py tests/test_flat_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_ivfq.log 2>&1 || { tail -30 gpurun_out/pytest_ivfq.log; exit 1; }
tail -1 gpurun_out/pytest_ivfq.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-forms > gpurun_out/bench_ivfq.json 2> gpurun_out/bench_ivfq.err || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"merge_ms": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/bench_ivfq.json
