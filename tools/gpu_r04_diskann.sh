#!/bin/bash
# r04: C4 DiskANN traversal (diskann_bfs) — batch-size sweep (traversals per CU) and PMC passes at nq 1024:
# SQ (wave cycles / parked / issue), FETCH_SIZE + clock, L2 hit/miss, TA/TD/TCP busy.  Each step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for nq in 1024 2048 4096; do
  timeout -k 10 240 python -u bench.py --workload diskann --nq $nq --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r04_diskann_nq$nq.json 2> gpurun_out/r04_diskann_nq$nq.err || { echo "diskann nq $nq failed"; tail -20 gpurun_out/r04_diskann_nq$nq.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04_diskann_nq$nq.json').read()); print($nq, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['recall_at_10'])"
done
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name="$1"; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --kernel-include-regex diskann_bfs --output-format csv \
      -d "$root/gpurun_out/pmc_r04_bfs_$name" -o run -- python3 "$root/bench.py" --workload diskann --no-cpu-baseline \
      --steps 2 --warmup 1 > "$root/gpurun_out/pmc_r04_bfs_$name.log" 2>&1 || { tail -5 "$root/gpurun_out/pmc_r04_bfs_$name.log"; exit 1; }
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU
run fetch FETCH_SIZE GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum
run tatd TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE
python3 "$root/tools/pmc_summary.py" diskann_bfs "$root/gpurun_out/pmc_r04_bfs_sq" "$root/gpurun_out/pmc_r04_bfs_fetch" \
    "$root/gpurun_out/pmc_r04_bfs_l2" "$root/gpurun_out/pmc_r04_bfs_tatd" | tee "$root/gpurun_out/pmc_r04_bfs_summary.txt"
