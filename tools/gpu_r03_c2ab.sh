#!/bin/bash
# r03: C2 (Flat L2 1M x 768, nq 1024) and Flat 10M — A/B of the bounded-pass split (HIPANN_FLAT_PASS_A: 1/x of each
# split in pass A, 0 = one pass) and the grid (HIPANN_FLAT_BF16_BLOCKS).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in 1000000 10000000; do
for v in "20 0" "10 0" "40 0" "0 0" "20 512" "10 512"; do
  set -- $v
  if [ "$2" = 0 ]; then unset HIPANN_FLAT_BF16_BLOCKS; else export HIPANN_FLAT_BF16_BLOCKS=$2; fi
  HIPANN_FLAT_PASS_A=$1 timeout -k 10 300 python3 bench.py --workload flat --n $n --no-cpu-baseline --no-alt-forms --no-suite \
      --no-c5 --steps 10 --warmup 2 > gpurun_out/c2ab.json 2> gpurun_out/c2ab.err || { tail -20 gpurun_out/c2ab.err; exit 1; }
  python3 - "n=$n passA=1/$1 blocks=$2" <<'PY'
import json, sys
for l in open('gpurun_out/c2ab.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"{sys.argv[1]:36s} {j['value']:9.1f} QPS  step {j['ms_per_step']:.3f} ms  kernel {r['kernel_ms']:.3f} ms  frac {r['frac']:.3f}")
PY
done
done
