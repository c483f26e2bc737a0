#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_diskann_gpu.py tests/test_configs_gpu.py -k "diskann or c4" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dk.log 2>&1 || { tail -30 gpurun_out/pytest_dk.log; exit 1; }
tail -1 gpurun_out/pytest_dk.log
HIPANN_LIB=tunelib/sq16.so timeout -k 10 300 python -u -m pytest tests/test_diskann_gpu.py tests/test_configs_gpu.py -k "diskann or c4" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dk16.log 2>&1 || { tail -30 gpurun_out/pytest_dk16.log; exit 1; }
tail -1 gpurun_out/pytest_dk16.log
tools/gpu_bfs_ab.sh
timeout -k 10 120 python -c "
import sys, json; sys.path.insert(0, 'duckdb-annsearch_amd'); sys.path.insert(0, '.')
import hipann, bench
r = bench.batch_distance_microbench(hipann)
for s in r['shapes']: print(s)
for s in r['break_even_sweep_d768']: print(s)
print('break_even', r['break_even_n_times_d'])
" > gpurun_out/bd_micro.log 2>&1; tail -20 gpurun_out/bd_micro.log
