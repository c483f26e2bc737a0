#!/usr/bin/env bash
# Flat bf16 pipeline depth A/B (HIPANN_B16_NB = 3, 4, 5): parity subset first, then the 10M / 1M lines.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for nb in 3 4 5; do
  HIPANN_B16_NB=$nb timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_flat_nb$nb.log 2>&1 || { tail -30 gpurun_out/pytest_flat_nb$nb.log; exit 1; }
  echo "NB=$nb $(tail -1 gpurun_out/pytest_flat_nb$nb.log)"
  for cfg in "10000000 l2" "1000000 l2"; do
    set -- $cfg
    HIPANN_B16_NB=$nb timeout -k 10 240 python bench.py --workload flat --n $1 --metric $2 --no-cpu-baseline --no-alt-forms --no-suite --steps 5 > gpurun_out/flatnb.json 2> gpurun_out/flatnb.err || { tail -5 gpurun_out/flatnb.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/flatnb.json')); r=d['roofline']
print('NB=$nb', '$1', '$2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('rerank_fallbacks_total'))"
  done
done
