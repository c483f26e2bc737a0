#!/bin/bash
# r06: C2 (Flat L2 1M x 768) seed-sample size A/B (HIPANN_FLAT_SAMPLE rows of the keys-mode seed pass; 16384 shipped),
# and Flat 10M at the same settings, same box, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
    for S in 16384 4096 8192 32768; do
        for N in 1000000 10000000; do
            HIPANN_FLAT_SAMPLE=$S timeout -k 10 300 python -u bench.py --workload flat --n $N --no-cpu-baseline --no-suite \
                --no-alt-forms --no-c5 --steps 10 --warmup 3 > gpurun_out/r06s_${S}_${N}_$rep.json 2> gpurun_out/r06s_${S}_${N}_$rep.err \
                || { tail -5 gpurun_out/r06s_${S}_${N}_$rep.err; exit 1; }
            python3 -c "import json; d=json.loads(open('gpurun_out/r06s_${S}_${N}_$rep.json').read()); r=d['roofline']; print('n=$N sample=$S', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('recall_at_10'), d.get('rerank_fallbacks'))"
        done
    done
done
