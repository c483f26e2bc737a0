#!/bin/bash
# r05: the extension's per-query IVF call (nq = 1) — kernel trace of the timed steps and its per-step breakdown.
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/nq1tr" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq 1 --steps 40 --warmup 5 \
    > "$root/gpurun_out/nq1tr.log" 2>&1 ) || { tail -5 gpurun_out/nq1tr.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/nq1tr.log | head -1
python3 tools/trace_summary.py gpurun_out/nq1tr ivf_scan_mfma_h 20
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open(next(__import__('pathlib').Path('gpurun_out/nq1tr').rglob('*kernel_trace.csv')))))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'ivf_scan_mfma_h' in r['Kernel_Name']]
a,b=idx[25],idx[26]
t0=int(rows[a]['Start_Timestamp'])
for r in rows[a:b+1]:
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    print(f"  {s:8.1f} {e:8.1f} {e-s:6.1f} {r['Kernel_Name'][:60]}")
PY
