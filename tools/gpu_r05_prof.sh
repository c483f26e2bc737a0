#!/bin/bash
# r05 profiles: kernel-trace/stats of the IVF headline step (per-step breakdown), of Flat 10M and of the C5 12.5M IP
# shard (int8 bounded passes), and one PMC pass (TA/TD busy, GRBM) on the Flat 10M kernel.
#   → gpurun_out/r05prof_{ivf,flat10m,c5ip}/, gpurun_out/r05prof_*.txt
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
o="$root/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/r05prof_ivf" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 5 \
    > "$o/r05prof_ivf.log" 2>&1 || { tail -5 "$o/r05prof_ivf.log"; exit 1; }
python3 "$root/tools/trace_summary.py" "$o/r05prof_ivf" ivf_scan_mfma_h 5 > "$o/r05prof_ivf_breakdown.txt" || exit 1
cat "$o/r05prof_ivf_breakdown.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/r05prof_flat10m" -o run -- \
    python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 10 --warmup 3 \
    > "$o/r05prof_flat10m.log" 2>&1 || { tail -5 "$o/r05prof_flat10m.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/r05prof_c5ip" -o run -- \
    python3 "$root/bench.py" --workload flat --n 12500000 --metric ip --no-cpu-baseline --no-alt-forms --no-suite \
    --no-c5 --steps 10 --warmup 3 > "$o/r05prof_c5ip.log" 2>&1 || { tail -5 "$o/r05prof_c5ip.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum \
    TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex flat_bf16_k64 --output-format csv \
    -d "$o/r05prof_flat10m_tatd" -o run -- python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms \
    --no-suite --no-c5 --steps 1 --warmup 0 > "$o/r05prof_flat10m_tatd.log" 2>&1 || { tail -5 "$o/r05prof_flat10m_tatd.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-include-regex flat_bf16_k64 --output-format csv \
    -d "$o/r05prof_flat10m_sq" -o run -- python3 "$root/bench.py" --workload flat --no-cpu-baseline --no-alt-forms \
    --no-suite --no-c5 --steps 1 --warmup 0 > "$o/r05prof_flat10m_sq.log" 2>&1 || { tail -5 "$o/r05prof_flat10m_sq.log"; exit 1; }
python3 "$root/tools/pmc_summary.py" flat_bf16_k64 "$o/r05prof_flat10m_tatd" "$o/r05prof_flat10m_sq" | tee "$o/r05prof_flat10m_pmc.txt"
for w in flat10m c5ip; do
  echo "== $w"; grep -h '"ms_per_step"' "$o/r05prof_$w.log" | tail -1 | cut -c1-300
  f=$(find "$o/r05prof_$w" -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -d, -f1-6
done
