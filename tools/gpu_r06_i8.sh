#!/bin/bash
# r06: the int8 IVF form (7, opt-in) — its GPU tests, then same-box A/B against form 6 on the SURVEY mixture
# (σ 0.8, nprobe 16 / 32) and on the headline line (HIPANN_IVF_FORM), alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests/test_ivf_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
        -k "${TEST_K:-7 or i8}" > gpurun_out/r06i8_tests.log 2>&1 || { tail -40 gpurun_out/r06i8_tests.log; exit 1; }
    tail -2 gpurun_out/r06i8_tests.log
fi
[ -n "$TESTS_ONLY" ] && exit 0
for rep in 1 2; do
    timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16,32 6,7 \
        > gpurun_out/r06i8_mix_$rep.log 2>&1 || { tail -5 gpurun_out/r06i8_mix_$rep.log; exit 1; }
    grep sigma gpurun_out/r06i8_mix_$rep.log
done
for rep in 1 2; do
    for F in 6 7; do
        HIPANN_IVF_FORM=$F timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms \
            --no-c5 --steps 20 --warmup 5 > gpurun_out/r06i8_ivf_${F}_$rep.json 2> gpurun_out/r06i8_ivf_${F}_$rep.err \
            || { tail -5 gpurun_out/r06i8_ivf_${F}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06i8_ivf_${F}_$rep.json').read()); r=d['roofline']; print('ivf form=$F', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'), d.get('ids_eq_cpu_path'))"
    done
done
