#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_diskann_gpu.py tests/test_configs_gpu.py -k "diskann or c4" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dk.log 2>&1 || { tail -30 gpurun_out/pytest_dk.log; exit 1; }
tail -1 gpurun_out/pytest_dk.log
HIPANN_LIB=tunelib/bulk2.so timeout -k 10 300 python -u -m pytest tests/test_diskann_gpu.py tests/test_configs_gpu.py -k "diskann or c4" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dkb2.log 2>&1 || { tail -30 gpurun_out/pytest_dkb2.log; exit 1; }
tail -1 gpurun_out/pytest_dkb2.log
tools/gpu_bfs_ab.sh
