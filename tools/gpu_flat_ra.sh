#!/usr/bin/env bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py -k "flat or c2" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_flat_ra.log 2>&1 || { tail -30 gpurun_out/pytest_flat_ra.log; exit 1; }
tail -1 gpurun_out/pytest_flat_ra.log
for e in "HIPANN_B16_RA=1" "HIPANN_B16_RA=0"; do
  for cfg in "10000000 l2" "1000000 l2" "10000000 ip"; do
    set -- $cfg
    env $e timeout -k 10 240 python bench.py --workload flat --n $1 --metric $2 --no-cpu-baseline --no-alt-forms --no-suite --steps 5 > gpurun_out/flatra.json 2> gpurun_out/flatra.err || { tail -5 gpurun_out/flatra.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/flatra.json')); r=d['roofline']
print('$e', '$1', '$2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('lds_fill',{}).get('achieved_tbps'), d.get('rerank_fallbacks_total'))"
  done
done
