#!/bin/bash
# r06: host-BFS thread count (HIPANN_BFS_THREADS; r06 also tried a distance prefetch, HIPANN_BFS_PF, no gain) — DiskANN GPU tests, then same-box A/B of the C4 host-BFS path with
# the phase split (HIPANN_BFS_PROF=1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_diskann_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r06p_dk_tests.log 2>&1 || { tail -30 gpurun_out/r06p_dk_tests.log; exit 1; }
tail -1 gpurun_out/r06p_dk_tests.log
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; taskset -pc $$ 2>/dev/null | cut -c1-200
for rep in 1 2; do for P in ${THREADS:-16 14 12}; do
    HIPANN_BFS_PROF=1 HIPANN_BFS_THREADS=$P timeout -k 10 300 python -u bench.py --workload diskann --n 1000000 --d 1536 --diskann-host-bfs \
        --no-cpu-baseline --no-suite --steps 3 --warmup 1 > gpurun_out/r06p_bfs_$P.json 2> gpurun_out/r06p_bfs_$P.err \
        || { tail -5 gpurun_out/r06p_bfs_$P.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06p_bfs_$P.json').read()); print('bfs threads=$P', d['value'], d['ms_per_step'], d.get('ids_eq_oracle_bfs'))"
    grep "hipann bfs" gpurun_out/r06p_bfs_$P.err | tail -2
done; done
