#!/usr/bin/env bash
# SQ / TCC counters of the Flat bf16 filter kernel (default: the 64-dim K-step kernel), one PMC pass per group.
#   tools/gpu_k64_pmc.sh [kernel-regex]  → gpurun_out/k64_pmc{1,2,3}/ + summary on stdout
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
re="${1:-flat_bf16_k64}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA" \
           "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE"; do
  i=$((i+1))
  rm -rf "$root/gpurun_out/k64_pmc$i"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$re" --output-format csv \
      -d "$root/gpurun_out/k64_pmc$i" -o run -- \
      python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 1 --warmup 0 \
      > "$root/gpurun_out/k64_pmc$i.log" 2>&1 || { tail -5 "$root/gpurun_out/k64_pmc$i.log"; exit 1; }
done
python3 - "$root/gpurun_out" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for p in glob.glob(sys.argv[1] + "/k64_pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:28s} {tot[k]:.4g} (dispatches {n[k]})")
PY
