#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py tests/test_ivf_gpu.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gate.log 2>&1 || { tail -30 gpurun_out/pytest_gate.log; exit 1; }
tail -1 gpurun_out/pytest_gate.log
timeout -k 10 300 python -c "
import sys, json, time; sys.path.insert(0, 'duckdb-annsearch_amd'); sys.path.insert(0, '.')
import hipann, bench
print(json.dumps(bench.flat_auto_gate(hipann), indent=0))
" > gpurun_out/gate.log 2>&1; cat gpurun_out/gate.log | tr -d '\n' | head -c 3000
