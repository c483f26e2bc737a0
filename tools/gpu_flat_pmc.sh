#!/usr/bin/env bash
# SQ counters of the split-bf16 Flat kernel (one PMC pass, 8 SQ counters) beside a short bench run.
#   tools/gpu_flat_pmc.sh   → gpurun_out/bench_flat.json, gpurun_out/flat_pmc/
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload flat --no-cpu-baseline --no-alt-forms --steps 3 --warmup 1 \
    > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.err || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/bench_flat.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex flat_gemm_topk_bf \
    --output-format csv -d "$root/gpurun_out/flat_pmc" -o run -- \
    python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms --steps 1 --warmup 0 \
    > "$root/gpurun_out/flat_pmc.log" 2>&1 || { tail -5 "$root/gpurun_out/flat_pmc.log"; exit 1; }
python3 - "$root/gpurun_out/flat_pmc" <<'PY'
import csv, glob, sys, collections
f = [p for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)]
tot = collections.defaultdict(float); n = collections.Counter()
for p in f:
    for r in csv.DictReader(open(p)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(k, tot[k], n[k])
PY
