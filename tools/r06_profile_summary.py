"""Agreement table of the r06 roofline evidence (tools/gpu_r06_prof.sh output under gpurun_out/): per configuration the
bench line's kernel time (HIP events on the launch stream), the rocprofv3 kernel-trace time of the same kernel per
search (every dispatch of one search summed: Flat runs a keys-mode seed pass and the planned bounded passes), their
ratio, the PMC FETCH_SIZE bytes per search against the algorithmic bytes, and the fractions both times give.
    python tools/r06_profile_summary.py [gpurun_out] > profiles/r06/roofline_agreement_r06.txt
"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "gpurun_out"
CFG = {  # cfg: (pmc key, kernel substring, group-start substring or None)
    "ivf": ("ivf_10000000x768", "ivf_scan_mfma_h", None),
    "flat10m": ("flat_10000000x768", "flat_bf16_k64", "flat_bf16_k64<true, true"),
    "c2": ("flat_1000000x768", "flat_bf16_k64", "flat_bf16_k64<true, true"),
    "c5": ("flat_12500000x768_ip", "flat_bf16_k64", "flat_bf16_k64<false, true"),
    "diskann": ("diskann_1000000x1536", "diskann_bfs", None),
}


def trace_per_search(cfg, kern, grp, skip=3):
    f = next((OUT / f"r06prof_{cfg}" / "stats").rglob("*kernel_trace.csv"))
    rows = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    if grp:
        groups, cur = [], None
        for r, t in zip(rows, dur):
            if grp in r["Kernel_Name"]:
                if cur is not None:
                    groups.append(cur)
                cur = 0.0
            if cur is not None:
                cur += t
        if cur is not None:
            groups.append(cur)
        vals = groups[skip:]
    else:
        vals = dur[skip:]
    return sum(vals) / len(vals), len(vals)


def line_of(cfg):
    for ln in open(OUT / f"r06prof_{cfg}_stats.log"):
        if ln.startswith("{") and '"ms_per_step"' in ln:
            return json.loads(ln)
    return None


def main():
    print("# r06 roofline evidence, one box, this tree (tools/gpu_r06_prof.sh): kernel-trace/stats pass and a separate")
    print("# rocprofv3 --pmc FETCH_SIZE pass per configuration; bytes = 2*1024*FETCH_SIZE (gfx950 correction)")
    print(f"{'config':9} {'kernel':20} {'line ms':>8} {'trace ms':>9} {'ratio':>6} {'n':>3} {'line frac':>9} "
          f"{'trace frac':>10} {'PMC GB':>7} {'alg GB':>7} {'PMC/alg':>7}")
    for cfg, (key, kern, grp) in CFG.items():
        try:
            ln = line_of(cfg)
            roof = ln["roofline"]
            tms, n = trace_per_search(cfg, kern, grp)
            pmc = json.loads((OUT / f"pmc_{key}.json").read_text())
        except Exception as e:  # noqa: BLE001
            print(f"{cfg:9} missing: {e!r}")
            continue
        lms = roof["kernel_ms"]
        frac_t = roof["frac"] * lms / tms
        alg = roof.get("algorithmic_per_launch_gb")
        tb = pmc["hbm_bytes_per_launch"] / 1e9
        print(f"{cfg:9} {roof['kernel'][:20]:20} {lms:8.3f} {tms:9.3f} {tms / lms:6.3f} {n:3d} {roof['frac']:9.4f} "
              f"{frac_t:10.4f} {tb:7.3f} {alg if alg else float('nan'):7.3f} {tb / alg if alg else float('nan'):7.3f}")


if __name__ == "__main__":
    main()
