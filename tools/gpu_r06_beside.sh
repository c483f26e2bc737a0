#!/bin/bash
# r06: host-BFS gathers enqueued beside the next group's phase (HIPANN_BFS_BESIDE) — DiskANN GPU tests, then same-box
# A/B of the C4 host-BFS path over CONFIGS (beside:groups), with the phase split (HIPANN_BFS_PROF=1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_diskann_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r06s_dk_tests.log 2>&1 || { tail -30 gpurun_out/r06s_dk_tests.log; exit 1; }
tail -1 gpurun_out/r06s_dk_tests.log
for rep in 1 2; do for C in ${CONFIGS:-0:2 1:2 1:3}; do
    B=${C%%:*}; G=${C##*:}
    HIPANN_BFS_PROF=1 HIPANN_BFS_BESIDE=$B HIPANN_BFS_GROUPS=$G timeout -k 10 300 python -u bench.py --workload diskann \
        --n 1000000 --d 1536 --diskann-host-bfs --no-cpu-baseline --no-suite --steps 3 --warmup 1 \
        > gpurun_out/r06s_bfs_${B}_$G.json 2> gpurun_out/r06s_bfs_${B}_$G.err || { tail -5 gpurun_out/r06s_bfs_${B}_$G.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06s_bfs_${B}_$G.json').read()); print('bfs beside=$B groups=$G', d['value'], d['ms_per_step'], d.get('recall_at_10'), d.get('ids_eq_oracle_bfs'))"
    grep "hipann bfs" gpurun_out/r06s_bfs_${B}_$G.err | tail -2
done; done
