#!/usr/bin/env python3
"""Per-dispatch averages of every PMC counter of the kernels matching a name, from rocprofv3 CSV dirs.
   python tools/pmc_summary.py <kernel-substring> <dir> [<dir> ...]"""
import collections, csv, glob, os, sys

kern = sys.argv[1]
for root in sys.argv[2:]:
    tot = collections.defaultdict(float)
    disp = set()
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add((f, r["Dispatch_Id"]))
    n = max(len(disp), 1)
    print(f"{root}: {len(disp)} dispatches")
    for k, v in sorted(tot.items()):
        print(f"  {k:28s} {v / n:16.4g}")
