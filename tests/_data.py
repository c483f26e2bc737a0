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


def check_topk_parity(xb, xq, D, I, Do, Io, metric=0, tau=1e-5, dist_rtol=1e-5, dist_atol=None, min_exact=0.99):
    """Parity rule: ids/order identical to the oracle except inside near-tie windows.

    For every rank where the labels differ, the exact (fp64) distances of the two labels must lie
    within ``tau * scale`` of each other (scale = |q|² + max |x|² for L2, |q|·max|x| for IP: the
    rounding scale of the fp32 forms), the returned label list must hold distinct valid labels, and
    at least ``min_exact`` of all slots must match exactly.  Reported distances must match the fp64
    distance of the returned label within dist_rtol (relative) / dist_atol (absolute, default from
    the scale).  Pads (-1) must coincide.
    """
    nq, k = I.shape
    assert I.shape == Io.shape
    pads = Io < 0
    assert np.array_equal(I < 0, pads), "pad slots differ"
    xmax = float(np.max(np.sum(xb.astype(np.float64) ** 2, 1))) if len(xb) else 0.0
    exact = (I == Io).mean() if I.size else 1.0
    assert exact >= min_exact, f"only {exact:.4f} of the slots match exactly"
    for qi in range(nq):
        q = xq[qi]
        qn = float(np.dot(q.astype(np.float64), q.astype(np.float64)))
        scale = (qn + xmax) if metric == 0 else np.sqrt(qn * xmax) * np.sqrt(xb.shape[1])
        atol = dist_atol if dist_atol is not None else 8e-6 * max(scale, 1e-30)
        valid = I[qi] >= 0
        labs = I[qi][valid]
        assert len(set(labs.tolist())) == len(labs), f"duplicate labels for query {qi}"
        if not len(labs):
            continue
        ex = O.exact_dists(xb, q, labs, metric)
        assert np.all(np.abs(D[qi][valid] - ex) <= atol + dist_rtol * np.abs(ex)), (
            f"query {qi}: distances off: {D[qi][valid]} vs exact {ex}")
        diff = np.nonzero(I[qi] != Io[qi])[0]
        if len(diff):
            eo = O.exact_dists(xb, q, Io[qi][diff], metric)
            eg = O.exact_dists(xb, q, I[qi][diff], metric)
            assert np.all(np.abs(eo - eg) <= tau * scale + 1e-12), (
                f"query {qi}: rank(s) {diff} differ beyond the tie window: {I[qi][diff]} vs {Io[qi][diff]}, "
                f"exact {eg} vs {eo}")
    # sortedness of the returned distances
    Dv = np.where(pads, np.nan, D)
    for qi in range(nq):
        v = Dv[qi][~np.isnan(Dv[qi])]
        if metric == 0:
            assert np.all(np.diff(v) >= 0), f"query {qi}: distances not ascending"
        else:
            assert np.all(np.diff(v) <= 0), f"query {qi}: distances not descending"
