#!/bin/bash
# Flat bf16 filter (form 4) check: GPU parity tests for Flat + configs, then the Flat 10M line and the C2
# sub-line under the 64-dim K-step kernel (default) and the 32-dim kernel (HIPANN_B16_K64=0), then a
# kernel trace of each so the filter's own duration is visible.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flat_gpu.py \
    tests/test_configs_gpu.py -m gpu > gpurun_out/flat_pytest.log 2>&1 || { tail -30 gpurun_out/flat_pytest.log; exit 1; }
tail -3 gpurun_out/flat_pytest.log
for v in "HIPANN_B16_K64=1" "HIPANN_B16_K64=0"; do
  echo "== [$v]"
  env $v timeout -k 10 300 python3 bench.py --workload flat --no-cpu-baseline --no-alt-forms --no-c5 --steps 10 \
      --warmup 3 > "gpurun_out/flat_$v.json" 2> "gpurun_out/flat_$v.err" || { tail -20 "gpurun_out/flat_$v.err"; exit 1; }
  python3 - "gpurun_out/flat_$v.json" <<'EOF'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); r = j.get('roofline', {})
        print(j['metric'], round(j['value']), j['ms_per_step'], r.get('achieved'), r.get('frac'))
        for name, s in (j.get('configs') or {}).items():
            print('  ', name, s.get('value'), s.get('ms_per_step'), (s.get('roofline') or {}).get('frac'))
EOF
done
cd /tmp && export TMPDIR=/tmp
for v in "HIPANN_B16_K64=1" "HIPANN_B16_K64=0"; do
  rm -rf "$root/gpurun_out/trace_$v"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/trace_$v" -o run -- \
      python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 5 \
      --warmup 2 > "$root/gpurun_out/trace_$v.log" 2>&1 || exit 1
  echo "== trace [$v]"
  f=$(ls "$root/gpurun_out/trace_$v"/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && head -6 "$f" | cut -c1-200
done
exit 0
