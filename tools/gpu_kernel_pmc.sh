#!/usr/bin/env bash
# PMC passes for one kernel of a bench workload, each counter set in its own rocprofv3 run (no trace
# domains beside --pmc; MI355X_MICROARCH.md slot limits: ≤ 8 SQ, ≤ 4 TCC with FETCH_SIZE = 3):
#   1. SQ: wave cycles, parked / issue-stall / active, MFMA busy, VALU / LDS instruction counts, LDS conflicts
#   2. FETCH_SIZE + GRBM_GUI_ACTIVE (HBM bytes, effective clock)
#   3. TCC_HIT_sum / TCC_MISS_sum (L2 hit rate)
#   tools/gpu_kernel_pmc.sh <tag> <kernel-regex> [bench args...]   → gpurun_out/pmc_<tag>_{sq,fetch,l2}/ + summary
set -uo pipefail
tag="$1"; kern="$2"; shift 2
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
    local name="$1"; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$kern" --output-format csv \
        -d "$root/gpurun_out/pmc_${tag}_$name" -o run -- python3 "$root/bench.py" --no-cpu-baseline --no-suite \
        --no-alt-forms --steps 2 --warmup 1 $BENCH_ARGS > "$root/gpurun_out/pmc_${tag}_$name.log" 2>&1 \
        || { tail -5 "$root/gpurun_out/pmc_${tag}_$name.log"; exit 1; }
}
BENCH_ARGS="$*"
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum
python3 "$root/tools/pmc_summary.py" "$kern" "$root/gpurun_out/pmc_${tag}_sq" "$root/gpurun_out/pmc_${tag}_fetch" \
    "$root/gpurun_out/pmc_${tag}_l2" | tee "$root/gpurun_out/pmc_${tag}_summary.txt"
