"""Test data helpers.

``mt19937_uniform`` reproduces, bit for bit, the inputs of the reference's GPU-vs-CPU tests:
``std::mt19937 rng(42); std::uniform_real_distribution<float> dist(-1, 1)`` filling the database
first and the queries second (faiss-metal/tests/test_metal_flat.mm:62-80, test_metal_ivfflat.mm:38-47),
as libstdc++ computes it: generate_canonical<float, 24> = float(u32) / 2^32 (clamped below 1), then
``u * (b - a) + a`` in float.  Verified against g++ in tests/test_oracle.py.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


def mt19937_uniform(count: int, seed: int = 42, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    bg = np.random.MT19937()
    bg._legacy_seeding(seed)
    u = bg.random_raw(count).astype(np.uint64)
    f = (u.astype(np.float32) / np.float32(4294967296.0)).astype(np.float32)
    f = np.where(f >= 1, np.nextafter(np.float32(1), np.float32(0)), f).astype(np.float32)
    return (f * np.float32(hi - lo) + np.float32(lo)).astype(np.float32)


def faiss_metal_case(nv: int, nq: int, d: int, seed: int = 42):
    """(xb, xq) exactly as the faiss-metal tests draw them."""
    a = mt19937_uniform(nv * d + nq * d, seed)
    return a[: nv * d].reshape(nv, d), a[nv * d:].reshape(nq, d)


def build_ivf_lists(xb: np.ndarray, centroids: np.ndarray, metric: int = 0):
    """Assign rows to their nearest centroid (FAISS IndexIVF::add: quantizer->assign, k = 1) and lay the
    lists out in CSR order (rows in insertion order within a list).  Returns (offsets, ids, codes)."""
    _, a = O.flat_search(centroids, xb, 1, metric)
    a = a[:, 0]
    nlist = centroids.shape[0]
    order = np.argsort(a, kind="stable")
    off = np.zeros(nlist + 1, np.int64)
    off[1:] = np.cumsum(np.bincount(a, minlength=nlist))
    return off, order.astype(np.int64), np.ascontiguousarray(xb[order])


# Parity rule: tau calibrated on the box (SURVEY §8c asks for 1e-6 "to be calibrated"); the observed
# gaps are collected in PARITY_STATS and written to gpurun_out/parity_calibration.json (conftest.py).
TAU = 1e-6
# The 2-term split forms (Flat form 2, IVF form 4: measurement only) drop terms worth up to 2^-15·‖q‖‖x‖
# per q·x (3·2^-16 plus the operands' 2^-17 remainders), i.e. ≤ 3.1e-5 of the L2 / IP scale.
SPLIT2_TAU = 4e-5
PARITY_STATS: list = []
PROBE_STATS: list = []  # oracle_on_gpu_probes: differing probe lists per check
CURRENT_TEST = None


def max_sqnorm(xb) -> float:
    """max_i ‖x_i‖² in fp64, chunked (1M × 768 rows would need a 6 GB fp64 copy at once)."""
    m = 0.0
    for r0 in range(0, len(xb), 65536):
        c = xb[r0:r0 + 65536].astype(np.float64)
        m = max(m, float(np.max(np.einsum("ij,ij->i", c, c))))
    return m


def check_probe_parity(cen, xq, P, Po, metric=0, tau=TAU):
    """IVF probe lists (coarse quantizer: a Flat search over the centroids) equal the oracle's, in order,
    except where the differing centroids are near ties at the nprobe boundary (fp64 distances within
    tau·scale).  Returns a bool mask of the queries whose probe lists are identical (the IVF results of
    the others may legitimately differ and are excluded from the id parity check)."""
    assert P.shape == Po.shape
    same = np.all(P == Po, axis=1)
    cmax = max_sqnorm(cen)
    for qi in np.nonzero(~same)[0]:
        q = xq[qi].astype(np.float64)
        w = tau * _scale(q, cmax, metric)
        lab_g, lab_o = P[qi], Po[qi]
        eg = O.exact_dists(cen, xq[qi], lab_g, metric)
        eo = O.exact_dists(cen, xq[qi], lab_o, metric)
        diff = np.nonzero(lab_g != lab_o)[0]
        assert np.all(np.abs(eg[diff] - eo[diff]) <= w + 1e-12), (
            f"query {qi}: probe lists differ beyond the tie window at ranks {diff}: {lab_g[diff]} vs {lab_o[diff]}")
    return same


def oracle_on_gpu_probes(oracle, cen, off, ids, codes, xq, k, P, Po, Do, Io, metric=0, tau=TAU):
    """The oracle's IVF answers held to the GPU's own probe lists.  Queries whose probe lists equal the oracle's keep
    the oracle's IndexIVFFlat::search results; a query whose list differs (only inside the coarse tie window:
    check_probe_parity asserts that) takes the oracle's IndexIVF::search_preassigned over the GPU's list — the scan
    the GPU ran — so the id parity check covers EVERY query of the batch instead of dropping those.  Returns
    (D, I, n_differing_probe_lists); the count is recorded in PARITY_STATS."""
    same = check_probe_parity(cen, xq, P, Po, metric, tau)
    D, I = Do.copy(), Io.copy()
    nd = int((~same).sum())
    if nd:
        Dp, Ip = oracle.ivf_search_preassigned(off, ids, codes, xq[~same], k, P[~same], metric)
        D[~same], I[~same] = Dp, Ip
    PROBE_STATS.append({"name": CURRENT_TEST, "probe_lists_differing": nd, "nq": int(len(xq)),
                        "queries": np.nonzero(~same)[0][:32].tolist()})
    return D, I, nd


def _scale(q64, xmax, metric):
    """Rounding scale of one query's fp32 distances: |q|² + max|x|² (L2) or |q|·max|x| (IP)."""
    qn = float(np.dot(q64, q64))
    return (qn + xmax) if metric == 0 else float(np.sqrt(qn * xmax))


def check_topk_parity(xb, xq, D, I, Do, Io, metric=0, tau=TAU, dist_rtol=1e-5, dist_tau=8e-6, min_exact=None,
                      name=None):
    """Parity rule: ids and order identical to the oracle's except inside near-tie windows.

    Per query, with w = tau·scale (scale = |q|² + max|x|² for L2, |q|·max|x| for IP — the rounding
    scale of the fp32 forms) and fp64 distances e(label):
      * at every rank where the labels differ, |e(gpu label) − e(oracle label)| ≤ w (a near tie);
      * the label SETS agree outside the boundary window: every label (of either list) whose key is
        below the oracle's k-th key − w is in both lists;
      * the returned labels are distinct and valid, pads (−1) coincide;
      * returned distances match the fp64 distance of the returned label within dist_rtol (relative)
        plus dist_tau·scale (absolute), and are sorted.
    The largest gap seen at a differing rank (in units of scale) is recorded in PARITY_STATS.
    Returns a dict of the observed statistics."""
    nq, k = I.shape
    assert I.shape == Io.shape
    pads = Io < 0
    assert np.array_equal(I < 0, pads), "pad slots differ"
    xmax = max_sqnorm(xb)
    exact = float((I == Io).mean()) if I.size else 1.0
    if min_exact is not None:
        assert exact >= min_exact, f"only {exact:.4f} of the slots match exactly"
    sgn = 1.0 if metric == 0 else -1.0  # key = dist (L2) or -ip (IP): ascending
    max_gap = 0.0
    ndiff = 0
    for qi in range(nq):
        q = xq[qi]
        scale = _scale(q.astype(np.float64), xmax, metric)
        w = tau * scale
        atol = dist_tau * max(scale, 1e-30)
        valid = I[qi] >= 0
        labs = I[qi][valid]
        assert len(set(labs.tolist())) == len(labs), f"duplicate labels for query {qi}"
        if not len(labs):
            continue
        eg = O.exact_dists(xb, q, labs, metric)
        assert np.all(np.abs(D[qi][valid] - eg) <= atol + dist_rtol * np.abs(eg)), (
            f"query {qi}: distances off: {D[qi][valid]} vs exact {eg}")
        olabs = Io[qi][valid]
        eo = O.exact_dists(xb, q, olabs, metric)
        diff = np.nonzero(labs != olabs)[0]
        if len(diff):
            ndiff += len(diff)
            gap = np.abs(eo[diff] - eg[diff])
            max_gap = max(max_gap, float(gap.max()) / max(scale, 1e-30))
            assert np.all(gap <= w + 1e-12), (
                f"query {qi}: rank(s) {diff} differ beyond the tie window (tau={tau}): {labs[diff]} vs "
                f"{olabs[diff]}, exact {eg[diff]} vs {eo[diff]}, gap/scale {gap / scale}")
            bound = sgn * eo[-1] - w
            inner_g = set(labs[sgn * eg < bound].tolist())
            inner_o = set(olabs[sgn * eo < bound].tolist())
            assert inner_g <= set(olabs.tolist()) and inner_o <= set(labs.tolist()), (
                f"query {qi}: label sets differ outside the boundary tie window")
    # sortedness of the returned distances
    Dv = np.where(pads, np.nan, D)
    for qi in range(nq):
        v = Dv[qi][~np.isnan(Dv[qi])]
        if metric == 0:
            assert np.all(np.diff(v) >= 0), f"query {qi}: distances not ascending"
        else:
            assert np.all(np.diff(v) <= 0), f"query {qi}: distances not descending"
    st = {"name": name or CURRENT_TEST, "nq": int(nq), "k": int(k), "d": int(xb.shape[1]) if xb.ndim == 2 else None,
          "n": int(len(xb)), "metric": int(metric), "exact_fraction": exact, "differing_slots": int(ndiff),
          "max_gap_over_scale": max_gap, "tau": tau}
    PARITY_STATS.append(st)
    return st
