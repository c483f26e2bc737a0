#!/bin/bash
# r04: the bounded Flat passes' count (flat_pass_plan; HIPANN_FLAT_PASSES pins it) at C2 (1M) and 10M x 768,
# after the Flat parity tests on the planned passes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_flat_kth_gpu.py tests/test_flat_gpu.py tests/test_request_k_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
    > gpurun_out/r04_passes_tests.log 2>&1 || { tail -30 gpurun_out/r04_passes_tests.log; exit 1; }
tail -1 gpurun_out/r04_passes_tests.log
fi
out=gpurun_out/passes_sweep_r04.txt
: > $out
for n in 1000000 10000000; do
  for P in ${PASSES_LIST:-auto 2 3 4 5}; do
    if [ "$P" = auto ]; then unset HIPANN_FLAT_PASSES; else export HIPANN_FLAT_PASSES=$P; fi
    timeout -k 10 300 python3 bench.py --workload flat --n $n --no-cpu-baseline --no-alt-forms \
        --steps 20 --warmup 3 > gpurun_out/passes_${n}_$P.log 2>&1 || { echo "n=$n P=$P failed"; tail -5 gpurun_out/passes_${n}_$P.log; exit 1; }
    echo "n=$n passes=$P $(grep -o '"value": [0-9.]*' gpurun_out/passes_${n}_$P.log | head -1) $(grep -o '"rerank_fallbacks": [0-9]*' gpurun_out/passes_${n}_$P.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/passes_${n}_$P.log | head -1)" | tee -a $out
  done
done
unset HIPANN_FLAT_PASSES
