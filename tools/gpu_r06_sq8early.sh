#!/bin/bash
# r06: the SQ8 id-gather's row loads issued before its visited-bit atomic returns (libhipann_sq8early.so,
# -DHIPANN_SQ8_EARLY=1) vs after (the default build) — DiskANN GPU tests on both builds, then same-box A/B of the
# C4 host-BFS path, alternating, with the phase split (HIPANN_BFS_PROF=1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/duckdb-annsearch_amd
for V in late early; do
    if [ $V = early ]; then LIB=$L/libhipann_sq8early.so; else LIB=$L/libhipann.so; fi
    HIPANN_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_diskann_gpu.py -m gpu -q -x --timeout 300 \
        --timeout-method thread > gpurun_out/r06e_dk_tests_$V.log 2>&1 || { tail -30 gpurun_out/r06e_dk_tests_$V.log; exit 1; }
    echo "$V: $(tail -1 gpurun_out/r06e_dk_tests_$V.log)"
done
for rep in 1 2; do for V in early late; do
    if [ $V = early ]; then LIB=$L/libhipann_sq8early.so; else LIB=$L/libhipann.so; fi
    HIPANN_LIB=$LIB HIPANN_BFS_PROF=1 timeout -k 10 300 python -u bench.py --workload diskann --n 1000000 --d 1536 \
        --diskann-host-bfs --no-cpu-baseline --no-suite --steps 3 --warmup 1 > gpurun_out/r06e_bfs_$V.json \
        2> gpurun_out/r06e_bfs_$V.err || { tail -5 gpurun_out/r06e_bfs_$V.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06e_bfs_$V.json').read()); print('bfs $V', d['value'], d['ms_per_step'], d.get('recall_at_10'))"
    grep "hipann bfs" gpurun_out/r06e_bfs_$V.err | tail -2
done; done
