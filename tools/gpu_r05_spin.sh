#!/bin/bash
# r05: polled host waits (HIPANN_SPIN_WAIT) A/B on one box: the Flat C2 device-API step (one host wait per search),
# the 10M step, and the DiskANN host-BFS batch (one wait per group step); then the Flat and DiskANN tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
line() { python -c "import json,sys; l=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=l['roofline']; print('$1', l['value'], l['ms_per_step'], r.get('kernel_ms'), r.get('frac'))"; }
for ab in HIPANN_SPIN_WAIT=0 HIPANN_SPIN_WAIT=1 HIPANN_SPIN_WAIT=0 HIPANN_SPIN_WAIT=1; do
  export "$ab"
  timeout -k 10 300 python -u bench.py --workload flat --n 1000000 --no-alt-forms --no-cpu-baseline --steps 40 --warmup 5 2>/dev/null | line "$ab C2" || exit 1
  tag=$(echo "$ab" | tr '=/' '__')
  timeout -k 10 300 python -u bench.py --workload diskann --diskann-host-bfs --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/spin_bfs_$tag.json 2> gpurun_out/spin_bfs_$tag.err || { tail -20 gpurun_out/spin_bfs_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/spin_bfs_$tag.json').read().strip().splitlines()[-1]); print('$ab bfs', d['value'], d['ms_per_step'], d.get('recall_at_10'))"
done
export HIPANN_SPIN_WAIT=1
timeout -k 10 300 python -u bench.py --workload flat --no-alt-forms --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | line "spin 10M" || exit 1
[ -n "${NO_TESTS:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "flat or c2 or c5 or diskann or bfs or c4 or harness or abi" \
    > gpurun_out/r05_spin_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05_spin_tests.log; exit $rc
