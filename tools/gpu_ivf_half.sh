#!/usr/bin/env bash
# IVF parity tests (incl. the C3-shape config test), then the IVF bench line without the suite.
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ivf_gpu.py tests/test_configs_gpu.py -k "ivf or c3" -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_ivfh.log 2>&1 || { tail -40 gpurun_out/pytest_ivfh.log; exit 1; }
tail -1 gpurun_out/pytest_ivfh.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-suite "$@" > gpurun_out/bench_ivfh.json 2> gpurun_out/bench_ivfh.err || { tail -20 gpurun_out/bench_ivfh.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_ivfh.json'))
r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'recall', d['recall_at_10'], 'kern', r['kernel_ms'], 'merge', r['merge_ms'], 'frac', r['frac'], 'fallbacks', d['ivf']['rerank_fallbacks_total'])
print(json.dumps(d.get('other_forms'), indent=0))"
