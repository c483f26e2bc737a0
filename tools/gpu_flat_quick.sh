#!/usr/bin/env bash
# Flat kernel iteration: Flat GPU tests (+ the C2 shape), then the 10M and 1M Flat lines.
#   tools/gpu_flat_quick.sh → gpurun_out/pytest_flat.log, gpurun_out/flat10m.json, gpurun_out/flat1m.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat_gpu.py tests/test_configs_gpu.py -k "flat or c2" -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_flat.log 2>&1 || { tail -40 gpurun_out/pytest_flat.log; exit 1; }
tail -2 gpurun_out/pytest_flat.log
for cfg in "flat10m --n 10000000" "flat1m --n 1000000" "flat10m_ip --n 10000000 --metric ip"; do
    set -- $cfg; name=$1; shift
    timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --no-suite --steps 10 --warmup 3 "$@" \
        > gpurun_out/$name.json 2> gpurun_out/$name.err || { tail -20 gpurun_out/$name.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', d['value'], 'qps', r['kernel_ms'], 'ms', r['frac'], 'frac', 'merge', r['merge_ms'], 'fallbacks', d.get('rerank_fallbacks_total'), {k: (v['queries_per_s'], v['ids_equal_to_reported_form']) for k, v in d.get('other_forms', {}).items()})"
done
