#!/bin/bash
# r06: the staggered int8 Flat schedule (HIPANN_K64_STAGGER, default on) — Flat GPU tests on it, then same-box A/B of
# the kernel time at 10M, C2 (1M) and C5 (12.5M IP), alternating 0/1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_flat_gpu.py tests/test_flat_kth_gpu.py tests/test_request_k_gpu.py \
    tests/test_configs_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06s_tests.log 2>&1 \
    || { tail -30 gpurun_out/r06s_tests.log; exit 1; }
tail -2 gpurun_out/r06s_tests.log
run() {  # tag, env value, bench args
    HIPANN_K64_STAGGER=$2 timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --no-suite --no-alt-forms \
        --no-c5 --steps 10 --warmup 3 ${@:3} > gpurun_out/r06s_$1_$2.json 2> gpurun_out/r06s_$1_$2.err \
        || { tail -5 gpurun_out/r06s_$1_$2.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06s_$1_$2.json').read()); r=d['roofline']; print('$1 stagger=$2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
}
for rep in 1 2; do
    for S in 0 1; do run f10m $S --n 10000000; done
done
for S in 0 1; do run c2 $S --n 1000000; done
for S in 0 1; do run c5 $S --n 12500000 --metric ip; done
