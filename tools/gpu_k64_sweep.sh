#!/usr/bin/env bash
# Flat bf16 filter throughput vs database size (HBM- vs MALL/L2-resident) and batch size: is the kernel
# latency-bound on its stream?  Prints TF/s (roofline.achieved) and kernel ms per configuration.
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
for cfg in "10000000 1024" "1000000 1024" "150000 1024" "2500000 4096" "10000000 4096" "10000000 2048"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --workload flat --n "$1" --nq "$2" --no-cpu-baseline --no-alt-forms --no-suite \
      --no-c5 --steps 5 --warmup 2 ${K64_EXTRA:-} > gpurun_out/sweep.json 2> gpurun_out/sweep.err \
      || { tail -20 gpurun_out/sweep.err; exit 1; }
  python3 - "$1" "$2" <<'EOF'
import json, sys
for l in open('gpurun_out/sweep.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"N={sys.argv[1]:>9} nq={sys.argv[2]:>5}  {r['achieved']:7.1f} TF/s  frac {r['frac']:.3f}  kernel {r['kernel_ms']:.3f} ms  step {j['ms_per_step']:.3f} ms")
EOF
done
