#!/usr/bin/env bash
# smoke(), the whole -m gpu suite and the default bench line (the round-end driver sequence).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_default.json')); r=d['roofline']
print('IVF', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['recall_at_10'], r.get('traffic'))
for k,v in d.get('configs',{}).items():
    print(k, v.get('value'), v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'), (v.get('roofline') or {}).get('traffic'), v.get('recall_at_10'), v.get('ids_equal_to_oracle'), v.get('error'))
"
