#!/bin/bash
# r05: C4 DiskANN host-BFS path (diskann_hip_search_batch), A/B over BFS_AB="VAR=a VAR=b" settings on one box, with
# the library's host-side split (HIPANN_BFS_PROF=1), then the DiskANN tests.  Stop at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for ab in ${BFS_AB:-DEFAULT=1}; do
  tag=$(echo "$ab" | tr '=/' '__')
  env "$ab" HIPANN_BFS_PROF=1 timeout -k 10 300 python -u bench.py --workload diskann --diskann-host-bfs --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/bfs_$tag.json 2> gpurun_out/bfs_$tag.err || { tail -20 gpurun_out/bfs_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bfs_$tag.json').read().strip().splitlines()[-1]); print('$ab', d['value'], d['ms_per_step'], d.get('recall_at_10'), d.get('ids_eq_oracle_bfs'))"
  grep "hipann bfs" gpurun_out/bfs_$tag.err | tail -2
done
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "diskann or bfs or c4" \
    > gpurun_out/r05_bfs_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_bfs_tests.log; exit $rc
