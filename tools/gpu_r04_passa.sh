#!/bin/bash
# r04: the bounded Flat passes' pass-A share (HIPANN_FLAT_PASS_A = 1/x of every split) at C2 (1M) and 10M x 768.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/passa_sweep_r04.txt
: > $out
for n in 1000000 10000000; do
  for pa in ${PASSA_LIST:-20 10 8 6 5 4}; do
    timeout -k 10 300 env HIPANN_FLAT_PASS_A=$pa python3 bench.py --workload flat --n $n --no-cpu-baseline --no-alt-forms \
        --steps 20 --warmup 3 > gpurun_out/passa_${n}_$pa.log 2>&1 || { echo "n=$n pa=$pa failed"; tail -5 gpurun_out/passa_${n}_$pa.log; exit 1; }
    echo "n=$n pass_a=1/$pa $(grep -o '"value": [0-9.]*' gpurun_out/passa_${n}_$pa.log | head -1) $(grep -o '"rerank_fallbacks": [0-9]*' gpurun_out/passa_${n}_$pa.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/passa_${n}_$pa.log | head -1)" | tee -a $out
  done
done
