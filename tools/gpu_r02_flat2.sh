#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py -k "flat or c2" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_flat2.log 2>&1 || { tail -30 gpurun_out/pytest_flat2.log; exit 1; }
tail -1 gpurun_out/pytest_flat2.log
tools/gpu_flat_ab.sh
