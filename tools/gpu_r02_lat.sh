#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ivf_gpu.py tests/test_flat_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1 || { tail -30 gpurun_out/pytest_lat.log; exit 1; }
tail -1 gpurun_out/pytest_lat.log
for nq in 1 4 1024; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq $nq --steps 20 > gpurun_out/ivf_nq$nq.json 2> gpurun_out/ivf_nq$nq.err || { tail -5 gpurun_out/ivf_nq$nq.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ivf_nq$nq.json')); r=d['roofline']
print('nq$nq', d['value'], d['ms_per_step'], r['kernel_ms'], r['merge_ms'], r['frac'], d['recall_at_10'])"
done
