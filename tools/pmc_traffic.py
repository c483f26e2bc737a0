#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from a rocprofv3 ``--pmc FETCH_SIZE`` pass.

MI355X_MICROARCH.md (§HBM, §rocprofv3 PMC slots) prescribes the recipe this follows:
  * FETCH_SIZE is collected in its own pass (it takes 3 of the 4 TCC slots; no WRITE_SIZE beside it,
    and no -s/-r/trace domains beside --pmc);
  * FETCH_SIZE is in KiB (counter_defs.yaml: (...)/1024), so bytes = 1024 · FETCH_SIZE;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read
    (128-B requests tallied at 64 B), so bytes are doubled before comparing with a byte count.

Usage:
  python tools/pmc_traffic.py <rocprofv3 -d dir> <kernel-name substring> [--skip N] [--out file.json]
The dispatches of the kernel (after skipping the first N, e.g. warm-up) are averaged.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys


def find_csv(root: str, suffix: str) -> list[str]:
    return sorted(glob.glob(os.path.join(root, "**", f"*{suffix}"), recursive=True))


def traffic(root: str, kernel: str, skip: int = 0, per_step: int = 1, group_start: str = None) -> dict:
    files = find_csv(root, "counter_collection.csv")
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    per_dispatch: dict[tuple, float] = {}
    names: dict[tuple, str] = {}
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != "FETCH_SIZE":
                    continue
                key = (f, int(row.get("Dispatch_Id", 0)))
                per_dispatch[key] = per_dispatch.get(key, 0.0) + float(row["Counter_Value"])
                names[key] = row.get("Kernel_Name", "")
    order = sorted(per_dispatch, key=lambda k: k[1])
    if group_start:
        # the kernel runs a varying number of times per search (Flat's keys-mode seed pass, then the planned bounded
        # passes): a search starts at each dispatch whose name contains group_start; groups are summed, the first
        # `skip` searches (warm-up) and a trailing partial group dropped
        groups, cur = [], None
        for k in order:
            if group_start in names[k]:
                if cur is not None:
                    groups.append(cur)
                cur = 0.0
            if cur is not None:
                cur += per_dispatch[k]
        vals = groups[skip:]
    else:
        vals = [per_dispatch[k] for k in order][skip * per_step:]
        # per_step > 1: the kernel runs that many times per search (e.g. Flat form 4's 64K-row threshold pre-pass
        # and the main scan); consecutive groups are summed so the figure is per search, like the bench's timer
        vals = [sum(vals[i:i + per_step]) for i in range(0, len(vals) - per_step + 1, per_step)]
    if not vals:
        raise SystemExit(f"no FETCH_SIZE rows for kernel '{kernel}' in {files}")
    kib = sum(vals) / len(vals)
    return {
        "kernel": kernel,
        "dispatches": len(vals),
        "dispatches_per_search": per_step,
        "fetch_size_kib_avg": kib,
        "hbm_bytes_per_launch": 2.0 * 1024.0 * kib,  # KiB → B, ×2 gfx950 correction (MI355X_MICROARCH.md §HBM)
        "recipe": "rocprofv3 --pmc FETCH_SIZE (own pass); bytes = 2 * 1024 * FETCH_SIZE",
    }


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("kernel")
    p.add_argument("--skip", type=int, default=0)
    p.add_argument("--per-step", type=int, default=1, help="dispatches of the kernel per search (summed)")
    p.add_argument("--group-start", help="kernel-name substring that opens each search's group of dispatches")
    p.add_argument("--name", help="the kernel name bench.py's roofline uses (default: the substring)")
    p.add_argument("--out")
    a = p.parse_args()
    res = traffic(a.dir, a.kernel, a.skip, a.per_step, a.group_start)
    if a.name:
        res["kernel"] = a.name
    if a.group_start:
        res["dispatches_per_search"] = f"grouped from each '{a.group_start}' dispatch"
    js = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js + "\n")
    print(js)


if __name__ == "__main__":
    sys.exit(main())
