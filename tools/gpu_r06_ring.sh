#!/bin/bash
# r06: the fp16 IVF scan's register-ring depth (MH_P super-steps in flight per wave) with one-term items: tuning builds
# libhipann_p4.so / libhipann_p8.so (make OUT=../libhipann_pN.so BUILD=build_pN EXTRA=-DHIPANN_MH_P=N) against the
# shipped library (MH_P 6), and libhipann_e0.so (HIPANN_MH_EARLY=0: the fill barrier before the first row loads), same
# box, alternating: the headline line and the SURVEY mixture.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$(pwd)/duckdb-annsearch_amd
for rep in 1 2; do
    for P in 6 4 8 e0; do
        if [ $P = 6 ]; then unset HIPANN_LIB; elif [ $P = e0 ]; then export HIPANN_LIB=$L/libhipann_e0.so; else export HIPANN_LIB=$L/libhipann_p$P.so; fi
        timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms --no-c5 --steps 20 \
            --warmup 5 > gpurun_out/r06p_ivf_${P}_$rep.json 2> gpurun_out/r06p_ivf_${P}_$rep.err \
            || { tail -5 gpurun_out/r06p_ivf_${P}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06p_ivf_${P}_$rep.json').read()); r=d['roofline']; print('ivf P=$P', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'))"
    done
done
for P in 6 4 8 e0; do
    if [ $P = 6 ]; then unset HIPANN_LIB; elif [ $P = e0 ]; then export HIPANN_LIB=$L/libhipann_e0.so; else export HIPANN_LIB=$L/libhipann_p$P.so; fi
    timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16 6 > gpurun_out/r06p_mix_$P.log 2>&1 \
        || { tail -5 gpurun_out/r06p_mix_$P.log; exit 1; }
    sed "s/^/P=$P /" gpurun_out/r06p_mix_$P.log | grep sigma | cut -c1-150
done
