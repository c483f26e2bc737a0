#!/usr/bin/env bash
# Flat bf16 filter A/B: bench --workload flat under HIPANN_K64_V variants given as arguments (default 0 1 2).
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
vs="${*:-0 1 2}"
for rep in 1 2; do
for v in $vs; do
  HIPANN_K64_V=$v timeout -k 10 300 python3 bench.py --workload flat --no-cpu-baseline --no-alt-forms --no-suite \
      --no-c5 --steps 10 --warmup 2 ${K64_EXTRA:-} > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { tail -20 gpurun_out/ab.err; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
for l in open('gpurun_out/ab.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"V={sys.argv[1]}  {r['achieved']:7.1f} TF/s  frac {r['frac']:.3f}  kernel {r['kernel_ms']:.3f} ms  step {j['ms_per_step']:.3f} ms")
PY
done
done
