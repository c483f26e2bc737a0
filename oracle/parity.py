"""Parity of a GPU top-k against the CPU path's top-k, as a report — TEST / MEASUREMENT INFRASTRUCTURE ONLY.

bench.py calls this in its cpu_baseline legs: the oracle's answers for the timed CPU sample (FAISS
IndexIVFFlat::search / IndexFlat::search restated in oracle.c, the extension's CPU path,
/root/reference/src/faiss_index.cpp:729-737) are compared with the GPU ids of the same queries.

The rule is tests/_data.py::check_topk_parity, restated without asserts so a bench line can carry
the outcome at full size:
  * ids and order identical, except at ranks where the two labels' fp64 distances lie within the tie window
    w = tau·scale (scale = ‖q‖² + max‖x‖² for L2, ‖q‖·max‖x‖ for IP; tau = 1e-6);
  * the label SETS agree below the oracle's k-th key − w;
  * pads coincide; returned labels are distinct;
  * returned distances within dist_rtol (relative) + dist_tau·scale of the fp64 distance of the returned label;
    where the ids agree, optionally within same_rtol of the oracle's own fp32 distance (both direct form: IVF).
"""
from __future__ import annotations

import numpy as np


def _exact(rows: np.ndarray, q: np.ndarray, metric: int) -> np.ndarray:
    r = rows.astype(np.float64)
    q = q.astype(np.float64)
    if metric == 0:
        t = r - q[None, :]
        return np.einsum("ij,ij->i", t, t)
    return r @ q


def topk_parity(rows_of, xq, D, I, Do, Io, metric: int, xmax2: float, tau: float = 1e-6, dist_rtol: float = 1e-5,
                dist_tau: float = 8e-6, same_rtol: float | None = None) -> dict:
    """rows_of(labels int64[m]) -> float32[m, d] (the database rows of those labels).  xmax2 = max‖x‖² over the
    database.  Returns the statistics and `parity_ok`; never raises on a mismatch (the violations are counted)."""
    nq, k = I.shape
    assert Io.shape == I.shape and D.shape == I.shape
    viol = {"pads": 0, "duplicates": 0, "distance": 0, "outside_window": 0, "set": 0, "order": 0, "same_id_distance": 0}
    max_gap = 0.0
    max_rel = 0.0
    max_same_rel = 0.0
    ndiff = 0
    qdiff = 0
    sgn = 1.0 if metric == 0 else -1.0
    for qi in range(nq):
        q = xq[qi]
        q64 = q.astype(np.float64)
        qn = float(q64 @ q64)
        scale = (qn + xmax2) if metric == 0 else float(np.sqrt(qn * xmax2))
        scale = max(scale, 1e-30)
        w = tau * scale
        if not np.array_equal(I[qi] < 0, Io[qi] < 0):
            viol["pads"] += 1
            continue
        valid = I[qi] >= 0
        labs, olabs = I[qi][valid], Io[qi][valid]
        if not len(labs):
            continue
        if len(set(labs.tolist())) != len(labs):
            viol["duplicates"] += 1
        eg = _exact(rows_of(labs), q, metric)
        err = np.abs(D[qi][valid] - eg)
        if np.any(err > dist_tau * scale + dist_rtol * np.abs(eg)):
            viol["distance"] += 1
        max_rel = max(max_rel, float(np.max(err / np.maximum(np.abs(eg), 1e-30))))
        dv = D[qi][valid]
        if np.any(np.diff(dv) < 0 if metric == 0 else np.diff(dv) > 0):
            viol["order"] += 1
        same = labs == olabs
        if same_rtol is not None and same.any():
            a, b = D[qi][valid][same].astype(np.float64), Do[qi][valid][same].astype(np.float64)
            rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
            max_same_rel = max(max_same_rel, float(rel.max()))
            if np.any(np.abs(a - b) > same_rtol * np.abs(b) + 1e-30):
                viol["same_id_distance"] += 1
        diff = np.nonzero(~same)[0]
        if len(diff):
            qdiff += 1
            ndiff += len(diff)
            eo = _exact(rows_of(olabs), q, metric)
            gap = np.abs(eo[diff] - eg[diff])
            max_gap = max(max_gap, float(gap.max()) / scale)
            if np.any(gap > w + 1e-12):
                viol["outside_window"] += 1
            bound = sgn * eo[-1] - w
            inner_g = set(labs[sgn * eg < bound].tolist())
            inner_o = set(olabs[sgn * eo < bound].tolist())
            if not (inner_g <= set(olabs.tolist()) and inner_o <= set(labs.tolist())):
                viol["set"] += 1
    ok = not any(viol.values())
    return {"queries": int(nq), "k": int(k), "ids_eq_cpu_path": round(float((I == Io).mean()), 6),
            "queries_identical": int(nq - qdiff), "differing_slots": int(ndiff),
            "max_gap_over_scale": max_gap, "tau": tau, "max_dist_rel_err_vs_fp64": max_rel,
            "max_dist_rel_vs_cpu_same_id": max_same_rel if same_rtol is not None else None,
            "violations": {k2: v for k2, v in viol.items() if v}, "parity_ok": ok}
