#!/bin/bash
# r06: the fp16 IVF scan's wide items (HIPANN_IVF_WIDE, default on) — IVF GPU tests on it, then same-box A/B of the
# SURVEY-mixture scan (σ 0.8, nprobe 16 / 32) and of the headline line, alternating over MODES (default 0 1;
# 2 = every item one-term); TEST_WIDE picks the mode the tests run under.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MODES=${MODES:-0 1}
if [ -z "$NO_TESTS" ]; then
    HIPANN_IVF_WIDE=${TEST_WIDE:-1} timeout -k 10 900 python -u -m pytest tests/test_ivf_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py \
        -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06w_tests.log 2>&1 \
        || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
    tail -2 gpurun_out/r06w_tests.log
fi
for rep in 1 2; do
    for W in $MODES; do
        HIPANN_IVF_WIDE=$W timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16,32 6 \
            > gpurun_out/r06w_mix_${W}_$rep.log 2>&1 || { tail -5 gpurun_out/r06w_mix_${W}_$rep.log; exit 1; }
        sed "s/^/wide=$W /" gpurun_out/r06w_mix_${W}_$rep.log | grep sigma
    done
done
for rep in 1 2; do
    for W in $MODES; do
        HIPANN_IVF_WIDE=$W timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms \
            --no-c5 --steps 20 --warmup 5 > gpurun_out/r06w_ivf_${W}_$rep.json 2> gpurun_out/r06w_ivf_${W}_$rep.err \
            || { tail -5 gpurun_out/r06w_ivf_${W}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06w_ivf_${W}_$rep.json').read()); r=d['roofline']; print('ivf wide=$W', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'), d.get('ids_eq_cpu_path'))"
    done
done
