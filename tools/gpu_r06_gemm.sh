#!/bin/bash
# r06: GEMM items for lists probed by more than 96 queries (HIPANN_IVF_GEMM, default on) — the IVF / C3 / request_k GPU
# tests on them first, then same-box A/B (alternating 0/1) of the SURVEY mixture probe (σ 0.8, nprobe 16 / 32), the
# headline line and the bench's mixture + intrinsic-dimension configurations.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests/test_ivf_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py tests/test_flat_gpu.py \
        -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06gm_tests.log 2>&1 \
        || { tail -40 gpurun_out/r06gm_tests.log; exit 1; }
    tail -2 gpurun_out/r06gm_tests.log
fi
for rep in 1 2; do
    for M in 0 1; do
        HIPANN_IVF_GEMM=$M timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16,32 6 \
            > gpurun_out/r06gm_mix_${M}_$rep.log 2>&1 || { tail -5 gpurun_out/r06gm_mix_${M}_$rep.log; exit 1; }
        sed "s/^/gemm=$M /" gpurun_out/r06gm_mix_${M}_$rep.log | grep sigma | cut -c1-170
    done
done
for rep in 1 2; do
    for M in 0 1; do
        HIPANN_IVF_GEMM=$M timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms \
            --no-c5 --steps 20 --warmup 5 > gpurun_out/r06gm_ivf_${M}_$rep.json 2> gpurun_out/r06gm_ivf_${M}_$rep.err \
            || { tail -5 gpurun_out/r06gm_ivf_${M}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06gm_ivf_${M}_$rep.json').read()); r=d['roofline']; print('ivf gemm=$M', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'))"
    done
done
for M in 0 1; do
    HIPANN_IVF_GEMM=$M timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-forms --no-c5 --steps 10 --warmup 3 \
        --only ivf_recall_vs_nprobe,C3_ivf_survey_mixture > gpurun_out/r06gm_suite_$M.json 2> gpurun_out/r06gm_suite_$M.err \
        || { tail -5 gpurun_out/r06gm_suite_$M.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06gm_suite_$M.json').read()); c=d['configs']
print('gemm=$M recall_vs_nprobe', c.get('ivf_recall_vs_nprobe'))
m=c.get('C3_ivf_survey_mixture', {}); print('gemm=$M mixture', {k: m.get(k) for k in ('value','ms_per_step','kernel_ms','frac','nprobe','parity_ok','ids_eq_cpu_path','flagged_per_batch')})"
done
