#!/bin/bash
# r06: IVF rows per work item (HIPANN_IVF_CH build switch: 2048 default, 1024 / 4096 tuning builds via HIPANN_LIB) —
# the IVF GPU tests on each build, then same-box A/B of the SURVEY mixture (σ 0.8, nprobe 16) and the headline line,
# alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=duckdb-annsearch_amd
for V in ${TESTV:-ch1024 ch4096}; do
    HIPANN_LIB=$PWD/$L/libhipann_$V.so timeout -k 10 600 python -u -m pytest tests/test_ivf_gpu.py -m gpu -q -x \
        --timeout 300 --timeout-method thread -k "not peer" > gpurun_out/r06c_tests_$V.log 2>&1 \
        || { tail -30 gpurun_out/r06c_tests_$V.log; exit 1; }
    echo "$V: $(tail -1 gpurun_out/r06c_tests_$V.log)"
done
for rep in 1 2; do
    for V in ${VARS:-default ch1024 ch4096}; do
        if [ $V = default ]; then LIB=$PWD/$L/libhipann.so; else LIB=$PWD/$L/libhipann_$V.so; fi
        HIPANN_LIB=$LIB timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16 6 \
            > gpurun_out/r06c_mix_${V}_$rep.log 2>&1 || { tail -5 gpurun_out/r06c_mix_${V}_$rep.log; exit 1; }
        sed "s/^/$V /" gpurun_out/r06c_mix_${V}_$rep.log | grep sigma
        HIPANN_LIB=$LIB timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms \
            --no-c5 --steps 20 --warmup 5 > gpurun_out/r06c_ivf_${V}_$rep.json 2> gpurun_out/r06c_ivf_${V}_$rep.err \
            || { tail -5 gpurun_out/r06c_ivf_${V}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06c_ivf_${V}_$rep.json').read()); r=d['roofline']; print('ivf $V', d['value'], d['ms_per_step'], r['kernel_ms'], r['merge_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'))"
        for NQ in ${SMALL_NQ:-}; do
            HIPANN_LIB=$LIB timeout -k 10 300 python -u bench.py --workload ivf --nq $NQ --no-cpu-baseline --no-suite \
                --no-alt-forms --no-c5 --steps 200 --warmup 20 > gpurun_out/r06c_nq${NQ}_${V}_$rep.json \
                2> gpurun_out/r06c_nq${NQ}_${V}_$rep.err || { tail -5 gpurun_out/r06c_nq${NQ}_${V}_$rep.err; exit 1; }
            python3 -c "import json; d=json.loads(open('gpurun_out/r06c_nq${NQ}_${V}_$rep.json').read()); print('ivf nq=$NQ $V', d['value'], d['ms_per_step'], d.get('recall_at_10'))"
        done
    done
done
