"""Per-step kernel breakdown from a rocprofv3 --kernel-trace csv: mean microseconds and launches per step,
a step being the window between consecutive launches of the step's anchor kernel (default: the IVF scan)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

path = Path(sys.argv[1])
anchor = sys.argv[2] if len(sys.argv) > 2 else "ivf_scan_mfma_h"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 5   # anchors skipped (warm-up); then 10 windows
f = next(path.rglob("*kernel_trace.csv"))
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
wins = list(zip(starts[skip:skip + 10], starts[skip + 1:skip + 11]))  # 10 anchor-to-anchor windows of the timed steps
tot = defaultdict(float)
cnt = defaultdict(int)
span = 0.0
for a, b in wins:
    span += (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    for r in rows[a:b]:
        name = r["Kernel_Name"].split("(")[0][:70]
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[name] += 1
n = len(wins)
print(f"{f}: {n} windows, mean step {span / n:.1f} us (anchor {anchor})")
busy = 0.0
for name, t in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {t / n:9.1f} us  x{cnt[name] / n:.1f}  {name}")
    busy += t / n
print(f"  {busy:9.1f} us  kernel-busy per step; gaps {span / n - busy:.1f} us")
