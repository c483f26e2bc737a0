#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
tools/gpu_ivf_ab.sh || exit 1
for nq in 256 512; do
  timeout -k 10 200 python bench.py --workload diskann --no-cpu-baseline --steps 10 --nq $nq > gpurun_out/bfs_nq$nq.json 2> gpurun_out/bfs_nq$nq.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/bfs_nq$nq.json')); r=d['roofline']
print('nq$nq', d['value'], r['kernel_ms_per_batch'], r['frac'], d['diskann']['bfs_steps_per_batch'])"
done
