#!/bin/bash
# r06: the fp16 IVF scan's round rotation (an item starts at the round another query group of its chunk last
# published): the IVF GPU tests with it, then same-box A/B, alternating — F = follow on (shipped), R = HIPANN_IVF_FOLLOW=0
# (runtime off), C = libhipann_f0.so (HIPANN_MH_FOLLOW=0: compiled out) — on the SURVEY mixture (σ 0.8, nprobe 16 / 32)
# and the headline, then the bench's intrinsic-dimension and mixture configurations for F and R.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$(pwd)/duckdb-annsearch_amd
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests/test_ivf_gpu.py tests/test_configs_gpu.py tests/test_request_k_gpu.py \
        -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r06f_tests.log 2>&1 \
        || { tail -40 gpurun_out/r06f_tests.log; exit 1; }
    tail -2 gpurun_out/r06f_tests.log
fi
setv() {
    unset HIPANN_LIB HIPANN_IVF_FOLLOW
    case $1 in R) export HIPANN_IVF_FOLLOW=0 ;; C) export HIPANN_LIB=$L/libhipann_f0.so ;; esac
}
for rep in 1 2; do
    for V in F R C; do
        setv $V
        timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16,32 6 > gpurun_out/r06f_mix_${V}_$rep.log 2>&1 \
            || { tail -5 gpurun_out/r06f_mix_${V}_$rep.log; exit 1; }
        sed "s/^/$V /" gpurun_out/r06f_mix_${V}_$rep.log | grep sigma | cut -c1-150
    done
done
for rep in 1 2; do
    for V in F R C; do
        setv $V
        timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms --no-c5 --steps 20 \
            --warmup 5 > gpurun_out/r06f_ivf_${V}_$rep.json 2> gpurun_out/r06f_ivf_${V}_$rep.err \
            || { tail -5 gpurun_out/r06f_ivf_${V}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06f_ivf_${V}_$rep.json').read()); r=d['roofline']; print('ivf $V', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'))"
    done
done
for V in F R; do
    setv $V
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-forms --no-c5 --steps 10 --warmup 3 \
        --only ivf_recall_vs_nprobe,C3_ivf_survey_mixture > gpurun_out/r06f_suite_$V.json 2> gpurun_out/r06f_suite_$V.err \
        || { tail -5 gpurun_out/r06f_suite_$V.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06f_suite_$V.json').read()); c=d['configs']
print('$V recall_vs_nprobe', c.get('ivf_recall_vs_nprobe'))
m=c.get('C3_ivf_survey_mixture', {}); print('$V mixture', {k: m.get(k) for k in ('value','ms_per_step','kernel_ms','frac','nprobe','flagged_per_batch')})"
done
unset HIPANN_LIB HIPANN_IVF_FOLLOW
[ -n "$NO_SAMPLE" ] || bash tools/gpu_r06_c2sample.sh
