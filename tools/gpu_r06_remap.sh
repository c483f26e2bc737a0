#!/bin/bash
# r06: the fp16 IVF scan's item → XCD mapping (HIPANN_IVF_REMAP: 1 = contiguous runs per XCD, a chunk's query groups on
# one L2; 0 = round-robin, the groups start together on different XCDs and share the Infinity Cache) — same-box A/B
# on the SURVEY mixture (σ 0.8, nprobe 16 / 32) and the headline line, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
    for R in 1 0; do
        HIPANN_IVF_REMAP=$R timeout -k 10 300 python -u tools/ivf_clustered_probe.py 0.8 10000000 16,32 6 \
            > gpurun_out/r06r_mix_${R}_$rep.log 2>&1 || { tail -5 gpurun_out/r06r_mix_${R}_$rep.log; exit 1; }
        sed "s/^/remap=$R /" gpurun_out/r06r_mix_${R}_$rep.log | grep sigma | cut -c1-140
    done
done
for rep in 1 2; do
    for R in 1 0; do
        HIPANN_IVF_REMAP=$R timeout -k 10 300 python -u bench.py --workload ivf --no-cpu-baseline --no-suite --no-alt-forms \
            --no-c5 --steps 20 --warmup 5 > gpurun_out/r06r_ivf_${R}_$rep.json 2> gpurun_out/r06r_ivf_${R}_$rep.err \
            || { tail -5 gpurun_out/r06r_ivf_${R}_$rep.err; exit 1; }
        python3 -c "import json; d=json.loads(open('gpurun_out/r06r_ivf_${R}_$rep.json').read()); r=d['roofline']; print('ivf remap=$R', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
    done
done
