#!/bin/bash
# r06: where the IVF scan's time goes on SURVEY §8(d)'s mixture (σ 0.8, nprobe 16: popular lists probed by up to ~400
# queries, so a list chunk is streamed once per ≤ 48-query group).  Kernel trace, FETCH_SIZE, SQ busy / MFMA / wait,
# L2 hit and TA / TD passes, each in its own run.  → gpurun_out/r06mix_*.{log,txt}
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
o="$root/gpurun_out"
K=ivf_scan_mfma_h
S=${MIX_SIGMA:-0.8}
NP=${MIX_NPROBE:-16}
P="python3 $root/tools/ivf_clustered_probe.py $S 10000000 $NP 6"
if [ -n "$MIX_BENCH" ]; then  # the bench's mixture configuration alone (its group-row and list statistics)
    (cd "$root" && timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-alt-forms --no-c5 --steps 5 --warmup 2 \
        --only C3_ivf_survey_mixture > "$o/r06mix_bench.json" 2> "$o/r06mix_bench.err") \
        || { echo "bench failed"; tail -5 "$o/r06mix_bench.err"; exit 1; }
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/r06mix_stats" -o run -- $P \
    > "$o/r06mix_stats.log" 2>&1 || { echo "stats failed"; tail -5 "$o/r06mix_stats.log"; exit 1; }
cat "$o/r06mix_stats.log"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$o/r06mix_fetch" -o run \
    -- $P > "$o/r06mix_fetch.log" 2>&1 || { echo "fetch failed"; tail -5 "$o/r06mix_fetch.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex "$K" --output-format csv \
    -d "$o/r06mix_sq" -o run -- $P > "$o/r06mix_sq.log" 2>&1 || { echo "sq failed"; tail -5 "$o/r06mix_sq.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-include-regex "$K" --output-format csv -d "$o/r06mix_tcc" -o run -- $P \
    > "$o/r06mix_tcc.log" 2>&1 || { echo "tcc failed"; tail -5 "$o/r06mix_tcc.log"; exit 1; }
python3 "$root/tools/pmc_summary.py" "$K" "$o/r06mix_fetch" "$o/r06mix_sq" "$o/r06mix_tcc" | tee "$o/r06mix_pmc.txt"
