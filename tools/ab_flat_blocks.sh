#!/usr/bin/env bash
# A/B of the bf16 Flat kernel's grid size (HIPANN_FLAT_BF16_BLOCKS) at 10M and 1M.
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"; mkdir -p gpurun_out
for b in 256 512 1024; do for n in 10000000 1000000; do
    HIPANN_FLAT_BF16_BLOCKS=$b timeout -k 10 200 python -u bench.py --workload flat --n $n --no-cpu-baseline --no-suite \
        --no-alt-forms --steps 10 --warmup 3 > gpurun_out/ab_${b}_${n}.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${b}_${n}.json').read().strip().splitlines()[-1]); r=d['roofline']
print('blocks $b n $n', d['value'], r['kernel_ms'], r['merge_ms'], d['rerank_fallbacks_total'])"
done; done
