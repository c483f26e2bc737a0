#!/bin/bash
# r06: host-BFS completion tokens (HIPANN_BFS_TOKEN) — DiskANN GPU tests, then same-box A/B of the C4 host-BFS path,
# then the IVF append probe at 10M (append + next search vs the search step).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_diskann_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r06b_dk_tests.log 2>&1 || { tail -30 gpurun_out/r06b_dk_tests.log; exit 1; }
tail -1 gpurun_out/r06b_dk_tests.log
for rep in 1 2; do for T in 0 1; do
    HIPANN_BFS_TOKEN=$T timeout -k 10 300 python -u bench.py --workload diskann --n 1000000 --d 1536 --diskann-host-bfs \
        --no-cpu-baseline --no-suite --steps 3 --warmup 1 > gpurun_out/r06b_bfs_$T.json 2> gpurun_out/r06b_bfs_$T.err \
        || { tail -5 gpurun_out/r06b_bfs_$T.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06b_bfs_$T.json').read()); print('bfs token=$T', d['value'], d['ms_per_step'], d.get('ids_eq_oracle_bfs'))"
done; done
PROBE_N=10000000 timeout -k 10 300 python -u tools/append_probe.py > gpurun_out/r06b_append.log 2>&1 || { tail -5 gpurun_out/r06b_append.log; exit 1; }
tail -1 gpurun_out/r06b_append.log | cut -c1-400
