#!/bin/bash
# r03: Flat form 4's second rerank of flagged queries — the Flat GPU tests, then the C5 shard line
# (12.5M x 768 IP: ≈2-3 flagged queries per batch) and Flat 10M L2.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_flat_gpu.py \
  > gpurun_out/candrr_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/candrr_tests.log; exit 1; }
tail -1 gpurun_out/candrr_tests.log
for args in "--n 12500000 --metric ip" "--n 10000000"; do
  timeout -k 10 300 python3 bench.py --workload flat $args --no-cpu-baseline --no-alt-forms --no-suite --no-c5 \
      --steps 10 --warmup 2 > gpurun_out/candrr.json 2> gpurun_out/candrr.err || { tail -20 gpurun_out/candrr.err; exit 1; }
  python3 - "$args" <<'PY'
import json, sys
for l in open('gpurun_out/candrr.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"{sys.argv[1]:28s} {j['value']:9.1f} QPS  step {j['ms_per_step']:.3f} ms  kernel {r['kernel_ms']:.3f} merge {r['merge_ms']:.3f} ms  frac {r['frac']:.3f}  fallbacks {j.get('rerank_fallbacks_total')}  oracle ids {j.get('ids_equal_to_oracle')}")
PY
done
