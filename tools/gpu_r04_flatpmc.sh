#!/bin/bash
# r04: PMC passes on the Flat int8 scan (flat_bf16_k64<I8>, 10M x 768 L2, nq 1024): MFMA busy, TD/TA busy, L1 pending
# stalls, LDS, FETCH_SIZE, L2 hits.  One counter group per pass, each under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name="$1"; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "flat_bf16_k64" --output-format csv \
      -d "$root/gpurun_out/pmc_r04_flat_$name" -o run -- python3 "$root/bench.py" --workload flat --no-cpu-baseline \
      --no-alt-forms --steps 1 --warmup 0 > "$root/gpurun_out/pmc_r04_flat_$name.log" 2>&1 \
      || { tail -5 "$root/gpurun_out/pmc_r04_flat_$name.log"; exit 1; }
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
run tatd TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE
run fetch FETCH_SIZE GRBM_COUNT
run l2 TCC_HIT_sum TCC_MISS_sum
python3 "$root/tools/pmc_summary.py" "flat_bf16_k64" "$root/gpurun_out/pmc_r04_flat_sq" "$root/gpurun_out/pmc_r04_flat_tatd" \
    "$root/gpurun_out/pmc_r04_flat_fetch" "$root/gpurun_out/pmc_r04_flat_l2" | tee "$root/gpurun_out/pmc_r04_flat_summary.txt"
