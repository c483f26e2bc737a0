"""Debug: Flat form 5 (int8 filter) against the fp32 form on several shapes; per-shape wrong-query counts,
fallback counters and the first wrong query's lists.  python tools/dbg_i8.py"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "duckdb-annsearch_amd"))
import hipann

for (n, d, nq, metric, dist) in [(1_000_000, 64, 512, 0, "n"), (1_000_000, 64, 512, 1, "n"), (1_000_000, 128, 512, 0, "n"),
                                 (1_000_000, 768, 512, 0, "u"), (600_000, 128, 256, 0, "n"), (1_000_000, 64, 256, 0, "n")]:
    rng = np.random.default_rng(11)
    if dist == "n":
        xb = rng.standard_normal((n, d), dtype=np.float32)
        xq = rng.standard_normal((nq, d), dtype=np.float32)
    else:
        xb = rng.uniform(-1, 1, (n, d)).astype(np.float32)
        xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    ix = hipann.HipIndexFlat(d, metric, xb)
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    out = {}
    for f in (4, 5):
        ix.form = f
        fb0 = ix.rerank_fallbacks()
        D1, I1 = ix.search(xq, 10)
        wrong = np.nonzero((I1 != I0).any(1))[0]
        out[f] = (len(wrong), ix.rerank_fallbacks() - fb0, ix.last_search_path())
        if f == 5 and len(wrong):
            q = wrong[0]
            print(f"  q{q} f5 D {D1[q][:5]} I {I1[q][:5]}\n      f0 D {D0[q][:5]} I {I0[q][:5]}", flush=True)
            print(f"  wrong queries (first 20): {wrong[:20].tolist()}", flush=True)
    print(f"n {n} d {d} nq {nq} metric {metric} {dist}: {out}", flush=True)
    ix.close()
