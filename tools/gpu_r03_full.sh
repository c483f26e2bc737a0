#!/bin/bash
# r03: the whole -m gpu suite, smoke and the default bench line (with its suite of config sub-lines).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_suite.log 2>&1 || { echo "suite failed"; tail -60 gpurun_out/r03_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03_bench.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r03_bench.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(j['metric'], round(j['value']), j['ms_per_step'], r.get('frac'), r.get('kernel_ms'))
        for name, s in (j.get('configs') or {}).items():
            print('  ', name, s.get('value'), s.get('ms_per_step'), (s.get('roofline') or {}).get('frac'))
PY
