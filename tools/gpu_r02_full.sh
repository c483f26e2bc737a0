#!/usr/bin/env bash
# Full -m gpu suite, then the default bench line (IVF + suite + C5) — round evidence.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_full.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_default.json')); r=d['roofline']
print('IVF', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['recall_at_10'])
for k,v in d.get('configs',{}).items():
    print(k, v.get('value'), v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'), v.get('error'))
"
