#!/usr/bin/env bash
# Flat bf16 filter: Flat + config GPU tests, then the Flat 10M line for the in-tree library (default
# schedule, one-pass A/B) and an optional reference library ($OLD_LIB).
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flat_gpu.py \
    tests/test_configs_gpu.py -m gpu > gpurun_out/flat_pytest.log 2>&1 || { tail -40 gpurun_out/flat_pytest.log; exit 1; }
tail -2 gpurun_out/flat_pytest.log
line() {
  timeout -k 10 300 python3 bench.py --workload flat --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 10 \
      --warmup 2 > gpurun_out/pa.json 2> gpurun_out/pa.err || { tail -20 gpurun_out/pa.err; return 1; }
  python3 - "$1" <<'PY'
import json, sys
for l in open('gpurun_out/pa.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"{sys.argv[1]:24s} {r['achieved']:7.1f} TF/s  frac {r['frac']:.3f}  kernel {r['kernel_ms']:.3f} ms  step {j['ms_per_step']:.3f} ms  QPS {j['value']:.0f}")
PY
}
for rep in 1 2; do
  line "default" || exit 1
  HIPANN_FLAT_PASS_A=0 line "one pass" || exit 1
  if [ -n "${OLD_LIB:-}" ]; then HIPANN_K64_V=1 HIPANN_LIB=$root/$OLD_LIB line "old lib" || exit 1; fi
done
