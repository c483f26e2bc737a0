#!/bin/bash
# r05: PMC passes on the IVF coarse key GEMM (flat_keys_bf3) inside the headline step: SQ wait / LDS / MFMA busy,
# then TA / TD / TCP stalls.  → gpurun_out/r05_keyspmc.txt
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
o="$root/gpurun_out"
K=${KEYS_KERNEL:-flat_keys_bf3}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "$K" --output-format csv \
    -d "$o/r05keys_sq" -o run -- python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 3 --warmup 1 \
    > "$o/r05keys_sq.log" 2>&1 || { tail -5 "$o/r05keys_sq.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum \
    TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$K" --output-format csv \
    -d "$o/r05keys_ta" -o run -- python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 3 --warmup 1 \
    > "$o/r05keys_ta.log" 2>&1 || { tail -5 "$o/r05keys_ta.log"; exit 1; }
python3 "$root/tools/pmc_summary.py" "$K" "$o/r05keys_sq" "$o/r05keys_ta" | tee "$o/r05_keyspmc.txt"
