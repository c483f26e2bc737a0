"""CPU tests of the oracle (the FAISS / DiskANN restatement used as the parity checker).

Pins the oracle to everything the reference itself provides for this path: the SQL known answers
(tests/golden/sql_known_answers.json, copied from test/sql/*.test) and the input generator of
faiss-metal's GPU-vs-CPU tests (std::mt19937(42)), plus internal consistency checks.
"""
from __future__ import annotations

import json
import shutil
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from _data import build_ivf_lists, faiss_metal_case, mt19937_uniform

GOLD = Path(__file__).resolve().parent / "golden"
SQL = json.loads((GOLD / "sql_known_answers.json").read_text())


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_mt19937_matches_libstdcxx(tmp_path):
    src = tmp_path / "mt.cpp"
    src.write_text('#include <random>\n#include <cstdio>\nint main(){std::mt19937 r(42);'
                   'std::uniform_real_distribution<float> d(-1.0f,1.0f);'
                   'for(int i=0;i<4096;i++) printf("%a\\n", d(r));}\n')
    exe = tmp_path / "mt"
    subprocess.run(["g++", "-O2", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    ref = np.array([float.fromhex(v) for v in out], np.float32)
    assert np.array_equal(ref, mt19937_uniform(4096))


def _flat_entries():
    return [(k, v) for k, v in SQL.items() if k.startswith(("faiss_basic", "edge_"))]


@pytest.mark.parametrize("name,case", _flat_entries())
def test_oracle_sql_known_answers_flat(oracle, name, case):
    xb = np.array(case["xb"], np.float32)
    deleted = set(case.get("deleted", []))
    for qc in case["queries"]:
        q = np.array([qc["q"]], np.float32)
        k = qc["k"]
        req = min(k + len(deleted), len(xb))  # FaissIndex::Search request_k (faiss_index.cpp:713-716)
        D, I = oracle.flat_search(xb, q, req, case["metric"])
        keep = [(d, i) for d, i in zip(D[0], I[0]) if i >= 0 and i not in deleted][:k]
        ids = [i for _, i in keep]
        dists = [d for d, _ in keep]
        if "ids" in qc:
            assert ids == qc["ids"][: len(ids)] and len(ids) == len(qc["ids"]), (ids, qc)
        if "dists" in qc:
            # ≤ 5 ulp: the reference printed 0.020000001 for |[1,0,0] − [0.9f,0.1f,0]|² whose exact
            # value is 0.0200000050664; the direct fp32 form gives 0.020000005 (Oracle).
            assert np.allclose(dists, qc["dists"], rtol=2.5e-7, atol=1e-9), (dists, qc["dists"])
        if "n_below_0.01" in qc:
            assert sum(d < 0.01 for d in dists) == qc["n_below_0.01"]
        if "n_results" in qc:
            assert len(ids) == qc["n_results"]


def test_oracle_sql_ivfflat_exact(oracle):
    case = SQL["faiss_ivfflat_exact"]
    xb = np.array(case["xb"], np.float32)
    cen = xb[[0, 4]].copy()  # any 2 centroids: nprobe = nlist makes the result exact
    off, ids, codes = build_ivf_lists(xb, cen)
    for qc in case["queries"]:
        D, I, P = oracle.ivf_search(cen, off, ids, codes, np.array([qc["q"]], np.float32), qc["k"], 2)
        assert I[0].tolist() == qc["ids"]
        if "dists" in qc:
            assert np.allclose(D[0], qc["dists"])


def test_oracle_pads_and_ties(oracle):
    xb = np.array([[1, 0], [1, 0], [0, 1]], np.float32)
    D, I = oracle.flat_search(xb, np.array([[1, 0]], np.float32), 5)
    assert I[0].tolist() == [0, 1, 2, -1, -1]  # tie → lower label first; pads (FLT_MAX, -1)
    assert D[0, 3] == np.finfo(np.float32).max
    D, I = oracle.flat_search(xb, np.array([[1, 0]], np.float32), 5, metric=1)
    assert I[0].tolist() == [0, 1, 2, -1, -1] and D[0, 3] == -np.finfo(np.float32).max
    # strict admission: a full heap keeps the earlier label on an exact tie at the boundary
    D, I = oracle.flat_search(xb, np.array([[1, 0]], np.float32), 1)
    assert I[0].tolist() == [0]


@pytest.fixture(scope="module", autouse=True)
def _golden_path():
    import sys
    sys.path.insert(0, str(GOLD))
    yield


def test_oracle_regression_flat(oracle):
    from make_golden import FLAT_CASES
    z = np.load(GOLD / "flat_mt19937.npz")
    for (nv, nq, d, k, m) in FLAT_CASES:
        xb, xq = faiss_metal_case(nv, nq, d)
        D, I = oracle.flat_search(xb, xq, k, m)
        key = f"flat_{nv}_{nq}_{d}_{k}_{m}"
        assert np.array_equal(I, z[key + "_I"]), key
        assert np.allclose(D, z[key + "_D"], rtol=1e-6, atol=1e-6), key


def test_oracle_regression_ivf(oracle):
    from make_golden import IVF_CASES
    z = np.load(GOLD / "ivf_mt19937.npz")
    for (nv, d, nlist, nprobe, nq, k, m) in IVF_CASES:
        xb, xq = faiss_metal_case(nv, nq, d)
        cen = np.ascontiguousarray(xb[:: nv // nlist][:nlist])
        off, ids, codes = build_ivf_lists(xb, cen, m)
        D, I, P = oracle.ivf_search(cen, off, ids, codes, xq, k, nprobe, m)
        key = f"ivf_{nv}_{d}_{nlist}_{nprobe}_{nq}_{k}_{m}"
        assert np.array_equal(P, z[key + "_P"]) and np.array_equal(I, z[key + "_I"]), key
        assert np.array_equal(off, z[key + "_off"])


def test_oracle_blas_vs_direct_forms_agree(oracle):
    """nq < 20 (direct) and nq >= 20 (norms + GEMM) must give the same neighbours up to near ties."""
    xb, xq = faiss_metal_case(3000, 40, 96)
    Db, Ib = oracle.flat_search(xb, xq, 10)          # BLAS form
    Dd = np.empty_like(Db)
    Id = np.empty_like(Ib)
    for s in range(0, 40, 10):
        Dd[s:s + 10], Id[s:s + 10] = oracle.flat_search(xb, xq[s:s + 10], 10)  # direct form
    assert (Ib == Id).mean() > 0.99
    assert np.allclose(Db, Dd, rtol=1e-4, atol=1e-4)


def test_oracle_ivf_full_probe_equals_flat(oracle):
    xb, xq = faiss_metal_case(2000, 10, 64)
    cen = np.ascontiguousarray(xb[::125][:16])
    off, ids, codes = build_ivf_lists(xb, cen)
    D, I, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 16)
    Df, If = oracle.flat_search(xb, xq, 10)  # nq < 20: same direct distance as the IVF scan
    assert np.array_equal(I, If)
    assert np.array_equal(D, Df)


def test_oracle_sq8_codec(oracle):
    z = np.load(GOLD / "sq8_qvectors.npz")
    xb = np.array(SQL["diskann_sq8_top1"]["xb"], np.float32)
    mins, scale = oracle.sq8_train(xb)
    codes = oracle.sq8_encode(xb, mins, scale)
    dec = oracle.sq8_decode(codes, mins, scale)
    assert np.array_equal(codes, z["codes"]) and np.array_equal(dec, z["decoded"])
    assert np.all(np.abs(dec - xb) <= scale / 255 / 2 + 1e-7)
    # constant dimension → scale 1 (provider.rs:187-190)
    m2, s2 = oracle.sq8_train(np.ones((3, 2), np.float32))
    assert s2.tolist() == [1.0, 1.0] and m2.tolist() == [1.0, 1.0]
    # rounding: half away from zero, clamped
    c = oracle.sq8_encode(np.array([[0.5 / 255], [2.0], [-1.0]], np.float32), np.array([0.0], np.float32),
                          np.array([1.0], np.float32))
    assert c[:, 0].tolist() == [1, 255, 0]


def test_oracle_sql_diskann_known_answers(oracle):
    case = SQL["diskann_batch"]
    xb = np.array(case["xb"], np.float32)
    n = len(xb)
    adj = np.array([[j for j in range(n) if j != i] for i in range(n)], np.uint32)  # complete graph
    qs = np.array([qc["q"] for qc in case["queries"]], np.float32)
    ids, dists, _ = oracle.diskann_search_batch(adj, [0], qs, 2, 8, vecs=xb)
    for i, qc in enumerate(case["queries"]):
        assert ids[i].tolist() == qc["ids"] and np.allclose(dists[i], qc["dists"])
    sq = SQL["diskann_sq8_top1"]
    xb = np.array(sq["xb"], np.float32)
    n = len(xb)
    adj = np.array([[j for j in range(n) if j != i] for i in range(n)], np.uint32)
    mins, scale = oracle.sq8_train(xb)
    codes = oracle.sq8_encode(xb, mins, scale)
    qs = np.array([qc["q"] for qc in sq["queries"]], np.float32)
    ids, _, _ = oracle.diskann_search_batch(adj, [0], qs, 3, 8, codes=codes, mins=mins, scale=scale)
    assert [r[0] for r in ids.tolist()] == [qc["top1"] for qc in sq["queries"]]


def test_oracle_bfs_regression_and_quality(oracle):
    z = np.load(GOLD / "bfs_2k.npz")
    a = mt19937_uniform(2000 * 32 + 20 * 32, seed=7)
    x, qs = a[: 2000 * 32].reshape(2000, 32), a[2000 * 32:].reshape(20, 32)
    ids, dists, st = oracle.diskann_search_batch(z["adj"], [0, 999], qs, 10, 48, vecs=x)
    assert np.array_equal(ids, z["ids"]) and np.array_equal(dists, z["dists"])
    assert [st["evals"], st["steps"]] == z["stats"].tolist()
    _, ex = oracle.flat_search(x, qs, 10)
    recall = np.mean([len(set(ids[i]) & set(ex[i])) / 10 for i in range(20)])
    assert recall > 0.8


def test_rust_binary_search_semantics():
    """The oracle's insert_result uses Rust's binary_search_by (std >= 1.82); restated in Python."""
    def bs(a, x):
        size, base = len(a), 0
        if size == 0:
            return 0
        while size > 1:
            half = size // 2
            mid = base + half
            base = base if a[mid] > x else mid
            size -= half
        if not (a[base] < x) and not (a[base] > x):
            return base
        return base + (1 if a[base] < x else 0)
    import bisect
    rng = np.random.default_rng(1)
    for _ in range(500):
        a = sorted(rng.integers(0, 20, rng.integers(0, 30)).tolist())
        x = int(rng.integers(-1, 21))
        p = bs(a, x)
        assert bisect.bisect_left(a, x) <= p <= bisect.bisect_right(a, x)


def test_diskann_file_roundtrip(tmp_path):
    import diskann_format as F
    x = mt19937_uniform(50 * 8).reshape(50, 8)
    adj = np.full((50, 4), 0xFFFFFFFF, np.uint32)
    adj[:, :3] = (np.arange(50)[:, None] + np.arange(1, 4)[None, :]) % 50
    mins, scale = x.min(0), x.max(0) - x.min(0)
    codes = np.round((x - mins) / scale * 255).clip(0, 255).astype(np.uint8)
    p = tmp_path / "t.diskann"
    F.write_index(p, x, adj, [0, 7], metric=1, build_complexity=64, sq8=(mins, scale, codes))
    f = F.open_index(p)
    assert (f.num_vectors, f.dimension, f.max_degree, f.metric, f.build_complexity) == (50, 8, 4, 1, 64)
    assert f.entry_points.tolist() == [0, 7]
    assert np.array_equal(f.vectors, x) and np.array_equal(f.adjacency, adj)
    assert f.neighbors(3).tolist() == [4, 5, 6]
    assert np.array_equal(f.sq8_codes, codes) and np.array_equal(f.sq8_min, mins)
    raw = p.read_bytes()
    (tmp_path / "bad.diskann").write_bytes(b"XANN" + raw[4:])
    with pytest.raises(ValueError, match="magic"):
        F.open_index(tmp_path / "bad.diskann")
    (tmp_path / "short.diskann").write_bytes(raw[:100])
    with pytest.raises(ValueError, match="too small"):
        F.open_index(tmp_path / "short.diskann")


def test_cpu_baseline_leg_runs():
    from oracle import cpu_baseline as CB
    xb, xq = faiss_metal_case(3000, 32, 64)
    qps, dt, nth = CB.flat_blas_qps(xb, xq, 10, 3000)
    assert qps > 0 and nth >= 1
    cen = np.ascontiguousarray(xb[::300][:10])
    off, ids, codes = build_ivf_lists(xb, cen)
    qps, dt, nth = CB.ivf_qps(cen, off, ids, codes, xq, 10, 4)
    assert qps > 0


def test_sq8_code_div255_fma_step_is_ieee():
    """diskann.hip sq8_value: code/255 as q0 = code·fl(1/255) and one fma residual step equals the IEEE
    fp32 quotient (Rust's `code as f32 / 255.0`, provider.rs:140-146) for every code 0..255 (fmas
    evaluated exactly with Fractions, then rounded once to fp32)."""
    from fractions import Fraction

    def rnd32(fr):
        c = np.float32(float(fr))  # nearest double, then nearest float: check the two neighbours exactly
        best = None
        for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
            err = abs(Fraction(float(cand)) - fr)
            even = (np.float32(cand).view(np.uint32) & 1) == 0
            if best is None or err < best[0] or (err == best[0] and even):
                best = (err, np.float32(cand))
        return best[1]

    r = np.float32(1.0) / np.float32(255.0)
    for code in range(256):
        q0 = np.float32(np.float32(code) * r)
        e = rnd32(Fraction(float(code)) - Fraction(float(q0)) * 255)
        a = rnd32(Fraction(float(e)) * Fraction(float(r)) + Fraction(float(q0)))
        assert a == np.float32(code) / np.float32(255.0), code


# ---- k-means restatement behind hipann_ivf_train (oracle_kmeans_train) ----
def _train_cases():
    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    from make_golden import TRAIN_CASES, train_data

    return TRAIN_CASES, train_data


def test_kmeans_oracle_matches_committed_fixture():
    """The committed ivf_train.npz (make_golden.py) is reproduced bit for bit: the restatement is deterministic
    given the seed (splitmix64 draws, integer D² weights, fp64 sums in row order)."""
    from oracle import oracle as O

    cases, train_data = _train_cases()
    z = np.load(Path(__file__).resolve().parent / "golden" / "ivf_train.npz")
    for name, metric, nlist, ts, niter, seed, init, dup in cases:
        cen, sizes = O.kmeans_train(train_data(dup), nlist, metric, ts, niter, seed, init)
        assert np.array_equal(cen, z[name + "_cen"]), name
        assert np.array_equal(sizes, z[name + "_sizes"]), name


def test_kmeans_oracle_semantics():
    """Stride sample of train_sample rows (faiss_index.cpp:307-313): the cluster sizes sum to train_sample;
    256 points per centroid at most; IP centroids are unit vectors (spherical); n < nlist is refused;
    k-means++ on 24 well-separated centres puts one centroid next to each."""
    from oracle import oracle as O

    cases, train_data = _train_cases()
    x = train_data(False)
    _, sizes = O.kmeans_train(x, 24, 0, 3000, 5, 1, 1)
    assert sizes.sum() == 3000
    _, sizes = O.kmeans_train(x, 8, 0, 0, 5, 1, 1)
    assert sizes.sum() == 256 * 8
    cen, _ = O.kmeans_train(x, 24, 1, 0, 5, 1, 1)
    assert np.allclose(np.linalg.norm(cen, axis=1), 1.0, atol=1e-6)
    with pytest.raises(ValueError):
        O.kmeans_train(x[:10], 24)
    # Lloyd lowers the k-means objective from the k-means++ start, and most true centres get their own centroid
    def inertia(c):
        _, a = O.flat_search(c, x, 1, 0)
        return float(((x - c[a[:, 0]]).astype(np.float64) ** 2).sum())

    c0, _ = O.kmeans_train(x, 24, 0, 0, 0, 1234, 1)
    cen, sizes = O.kmeans_train(x, 24, 0, 0, 25, 1234, 1)
    assert inertia(cen) < inertia(c0) and (sizes > 0).all()
    true = mt19937_uniform(24 * 48, seed=11).reshape(24, 48) * np.float32(3.0)
    d = ((cen[:, None, :] - true[None, :, :]) ** 2).sum(-1)
    assert len(set(d.argmin(1).tolist())) >= 22


def test_bench_parity_report_agrees_with_the_test_rule():
    """oracle/parity.py (the bench line's ids_eq_cpu_path / parity_ok) restates tests/_data.check_topk_parity without
    asserts: on the oracle's own answers, and on answers with an exact-tie swap, it reports parity_ok like the test
    rule passes; a swap beyond the tie window and a wrong distance are counted as violations."""
    from oracle import oracle as O
    from oracle.parity import topk_parity
    from _data import check_topk_parity, max_sqnorm

    xb, xq = faiss_metal_case(4000, 24, 32)
    xb = xb.copy()
    xb[7] = xb[3]  # an exact duplicate: its rank order is a tie
    D, I = O.flat_search(xb, xq, 10)
    xm = max_sqnorm(xb)
    rows = lambda labs: xb[labs]  # noqa: E731
    r = topk_parity(rows, xq, D, I, D, I, 0, xm)
    assert r["parity_ok"] and r["ids_eq_cpu_path"] == 1.0 and r["queries_identical"] == 24
    check_topk_parity(xb, xq, D, I, D, I)
    # a query whose answer contains the duplicate pair: swap them (inside the window)
    Dq, Iq = O.flat_search(xb, xb[3:4] + np.float32(1e-3), 10)
    I2 = Iq.copy()
    a, b = list(I2[0]).index(3), list(I2[0]).index(7)
    I2[0, a], I2[0, b] = I2[0, b], I2[0, a]
    r = topk_parity(rows, xb[3:4] + np.float32(1e-3), Dq, I2, Dq, Iq, 0, xm)
    assert r["parity_ok"] and r["differing_slots"] == 2
    # beyond the window: swap ranks 0 and 9 of query 0
    I3 = I.copy()
    I3[0, 0], I3[0, 9] = I3[0, 9], I3[0, 0]
    r = topk_parity(rows, xq, D, I3, D, I, 0, xm)
    assert not r["parity_ok"] and r["violations"].get("outside_window", 0) >= 1
    with pytest.raises(AssertionError):
        check_topk_parity(xb, xq, D, I3, D, I)
    D4 = D.copy()
    D4[1, 2] *= 1.01
    r = topk_parity(rows, xq, D4, I, D, I, 0, xm, same_rtol=2e-6)
    assert not r["parity_ok"] and r["violations"]["distance"] == 1 and r["violations"]["same_id_distance"] == 1


def test_ivf_search_preassigned_equals_search_on_its_own_probes():
    """IndexIVF::search = coarse step + search_preassigned: the restated search_preassigned on the oracle's own probe
    lists returns the oracle's IndexIVFFlat::search results bit for bit (the tests then hold the GPU scan to it on the
    GPU's probe lists when a list differs inside the coarse tie window)."""
    from oracle import oracle as O
    xb, xq = faiss_metal_case(4000, 30, 24)
    cen = np.ascontiguousarray(xb[::200][:20])
    for metric in (0, 1):
        off, ids, codes = build_ivf_lists(xb, cen, metric)
        D, I, P = O.ivf_search(cen, off, ids, codes, xq, 10, 5, metric)
        D2, I2 = O.ivf_search_preassigned(off, ids, codes, xq, 10, P, metric)
        assert np.array_equal(I, I2) and np.array_equal(D, D2)
        P2 = P.copy()
        P2[:, 0] = -1  # a skipped probe (-1) is not scanned
        D3, I3 = O.ivf_search_preassigned(off, ids, codes, xq, 10, P2, metric)
        D4, I4, _ = O.ivf_search(cen, off, ids, codes, xq, 10, 5, metric)
        assert not np.array_equal(I3, I4)
