#!/usr/bin/env bash
# DiskANN GPU tests, the C4 bench line, and (if tune/libhipann_prof.so exists) the per-phase cycle profile.
#   tools/gpu_bfs_check.sh   → gpurun_out/pytest_diskann.log, gpurun_out/bench_diskann.json, gpurun_out/prof.err
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_diskann_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_diskann.log 2>&1 || { tail -30 gpurun_out/pytest_diskann.log; exit 1; }
tail -1 gpurun_out/pytest_diskann.log
timeout -k 10 200 python bench.py --workload diskann --no-cpu-baseline > gpurun_out/bench_diskann.json 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms_per_batch": [0-9.]*\|"recall_at_10": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_diskann.json
if [ -e tune/libhipann_prof.so ]; then
    HIPANN_LIB=tune/libhipann_prof.so timeout -k 10 200 python bench.py --workload diskann --no-cpu-baseline --steps 3 \
        --warmup 1 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit 1
    grep bfs-prof gpurun_out/prof.err | tail -1
fi
