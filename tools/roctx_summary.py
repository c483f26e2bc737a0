"""Summary of the library's roctx ranges (HIPANN_ROCTX=1) from a rocprofv3 --marker-trace --kernel-trace CSV directory:
per range name its count and mean / total host span, and per kernel its count and mean duration, so the stage spans
and the kernels they enqueue can be read side by side.
    python tools/roctx_summary.py <rocprofv3 output dir>
"""
from __future__ import annotations

import collections
import csv
import sys
from pathlib import Path


def rows(root: Path, suffix: str):
    for f in root.rglob(f"*{suffix}"):
        yield from csv.DictReader(open(f))


def main():
    root = Path(sys.argv[1])
    spans = collections.defaultdict(list)
    cols = None
    for r in rows(root, "marker_api_trace.csv"):
        cols = cols or list(r.keys())
        name = r.get("Function") or r.get("Name") or r.get("Message") or "?"
        try:
            spans[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        except (KeyError, ValueError):
            continue
    print(f"# marker columns: {cols}")
    print(f"{'range':36} {'count':>6} {'mean us':>10} {'total ms':>10}")
    for name, v in sorted(spans.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:36]:36} {len(v):6d} {sum(v) / len(v):10.2f} {sum(v) / 1e3:10.3f}")
    kern = collections.defaultdict(list)
    for r in rows(root, "kernel_trace.csv"):
        kern[r["Kernel_Name"].split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"\n{'kernel':60} {'count':>6} {'mean us':>10}")
    for name, v in sorted(kern.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"{name:60} {len(v):6d} {sum(v) / len(v):10.2f}")


if __name__ == "__main__":
    main()
