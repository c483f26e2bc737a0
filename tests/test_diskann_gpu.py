"""GPU parity tests of the DiskANN batch-distance bridge (include/hip_diskann_bridge.h) and of the
lock-step BFS over the HBM-resident id-gather path, against the oracle (distance.rs / ann_search.cpp
ComputeDistancesCPU / provider.rs SQ8 / disk_provider.rs search_batch restatements).

Tolerance (north_star: distances elementwise within 1e-5 relative): |gpu − cpu| ≤ 1e-5·|cpu| + a
summation-order term 2e-6·Σ|terms| (the reference's own CPU (sequential) and Metal (lane-strided)
sums differ in order too).
"""
from __future__ import annotations

import json
import threading
from pathlib import Path

import numpy as np
import pytest

from _data import mt19937_uniform

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
SQL = json.loads((GOLD / "sql_known_answers.json").read_text())


def close(out, ref, q, c, metric):
    terms = np.abs(q * c).sum(-1) if metric == 1 else ((q - c) ** 2).sum(-1)
    return np.all(np.abs(out - ref) <= 1e-5 * np.abs(ref) + 2e-6 * terms + 1e-30)


@pytest.mark.parametrize("n,d", [(1, 1), (7, 3), (64, 128), (64, 768), (128, 1536), (512, 1536), (1024, 768),
                                 (3000, 100)])
@pytest.mark.parametrize("metric", [0, 1])
def test_batch_distances(gpu, oracle, n, d, metric):
    rng = np.random.default_rng(n * 131 + d)
    q = rng.uniform(-1, 1, d).astype(np.float32)
    c = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    out = np.full(n, np.nan, np.float32)
    assert gpu.diskann_hip_batch_distances(q, c, n, d, metric, out) == 0
    ref = oracle.batch_distances(q, c, metric)
    assert close(out, ref, q[None], c, metric)
    out2 = np.full(n, np.nan, np.float32)   # reference symbol name, same code
    L = gpu.lib()
    fp = lambda a: a.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_float))  # noqa: E731
    assert L.diskann_metal_batch_distances(fp(q), fp(c), n, d, metric, fp(out2)) == 0
    assert np.array_equal(out, out2)


@pytest.mark.parametrize("metric", [0, 1])
def test_multi_batch_distances(gpu, oracle, metric):
    rng = np.random.default_rng(5)
    nq, d, tot = 50, 1536, 3200
    qs = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    c = rng.uniform(-1, 1, (tot, d)).astype(np.float32)
    qm = np.sort(rng.integers(0, nq, tot)).astype(np.uint32)
    out = np.empty(tot, np.float32)
    assert gpu.diskann_hip_multi_batch_distances(qs, c, qm, tot, nq, d, metric, out) == 0
    ref = oracle.multi_batch_distances(qs, c, qm, metric)
    assert close(out, ref, qs[qm], c, metric)
    # unsorted query_map works the same
    perm = rng.permutation(tot)
    out2 = np.empty(tot, np.float32)
    assert gpu.diskann_hip_multi_batch_distances(qs, c[perm], qm[perm], tot, nq, d, metric, out2) == 0
    assert np.array_equal(out2, out[perm])


def test_bridge_errors(gpu):
    q = np.zeros((2, 8), np.float32)
    c = np.zeros((4, 8), np.float32)
    out = np.zeros(4, np.float32)
    qm = np.array([0, 1, 2, 0], np.uint32)  # 2 >= nq
    assert gpu.diskann_hip_multi_batch_distances(q, c, qm, 4, 2, 8, 0, out) == -1
    assert gpu.diskann_hip_batch_distances(q[0], c, 4, 8, 7, out) == -1
    assert gpu.diskann_hip_available() == 1 and gpu.is_hip_available()


def test_wrappers_gate_and_succeed(gpu, oracle):
    rng = np.random.default_rng(9)
    d = 1536
    q = rng.uniform(-1, 1, d).astype(np.float32)
    small = rng.uniform(-1, 1, (8, d)).astype(np.float32)   # 12288 < MIN_GPU_WORK → declined
    assert not gpu.hip_batch_distances(q, small, 8, d, 0, np.empty(8, np.float32))
    assert gpu.MIN_GPU_WORK == 786432
    big = rng.uniform(-1, 1, (600, d)).astype(np.float32)   # 921600 ≥ MIN_GPU_WORK (DMA path: > 1 MiB)
    out = np.empty(600, np.float32)
    assert gpu.hip_batch_distances(q, big, 600, d, 0, out)
    assert close(out, oracle.batch_distances(q, big, 0), q[None], big, 0)


def test_bridge_thread_safety(gpu, oracle):
    rng = np.random.default_rng(11)
    d = 768
    qs = [rng.uniform(-1, 1, d).astype(np.float32) for _ in range(8)]
    cs = [rng.uniform(-1, 1, (300 + 37 * t, d)).astype(np.float32) for t in range(8)]
    outs = [np.empty(len(c), np.float32) for c in cs]
    rcs = [None] * 8

    def run(t):
        for _ in range(20):
            rcs[t] = gpu.diskann_hip_batch_distances(qs[t], cs[t], len(cs[t]), d, 0, outs[t])

    ts = [threading.Thread(target=run, args=(t,)) for t in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for t in range(8):
        assert rcs[t] == 0
        assert close(outs[t], oracle.batch_distances(qs[t], cs[t], 0), qs[t][None], cs[t], 0)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("d", [1536, 100])
def test_ids_gather_f32_and_sq8(gpu, oracle, fmt, metric, d):
    rng = np.random.default_rng(fmt * 10 + metric + d)
    N, nq, tot = 30000, 40, 5000
    x = rng.uniform(-1, 1, (N, d)).astype(np.float32)
    qs = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    ids = rng.integers(0, N, tot).astype(np.uint32)
    qm = np.sort(rng.integers(0, nq, tot)).astype(np.uint32)
    if fmt == 0:
        db = gpu.DiskannDeviceDB(x, 0)
        ref = oracle.multi_batch_distances(qs, x[ids], qm, metric)
        dec = x[ids]
    else:
        mins, scale = oracle.sq8_train(x)
        codes = oracle.sq8_encode(x, mins, scale)
        db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
        ref = oracle.sq8_distances_ids(qs, codes, mins, scale, ids, qm, metric)
        dec = oracle.sq8_decode(codes[ids], mins, scale)
    out = db.distances_ids(qs, ids, qm, metric)
    assert close(out, ref, qs[qm], dec, metric)
    with pytest.raises(gpu.HipAnnError):
        db.distances_ids(qs, np.array([N], np.uint32), np.array([0], np.uint32), metric)


@pytest.mark.parametrize("d", [1536, 100])
def test_sq8_decode_bit_identical(gpu, oracle, d):
    """The id-gather kernels dequantise exactly as provider.rs:140-146, (code as f32 / 255.0) * scale + min:
    with one-hot IP queries the distance of row r to e_j is exactly −v[r, j], compared bitwise with the
    oracle's decode (the same expression in C, -ffp-contract=off)."""
    rng = np.random.default_rng(d)
    N = 2000
    x = (rng.standard_normal((N, d)) * rng.uniform(0.1, 30, d)).astype(np.float32)
    mins, scale = oracle.sq8_train(x)
    codes = oracle.sq8_encode(x, mins, scale)
    db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
    dims = np.arange(0, d, 7)
    qs = np.zeros((len(dims), d), np.float32)
    qs[np.arange(len(dims)), dims] = 1.0
    rows = rng.integers(0, N, 300).astype(np.uint32)
    ids = np.tile(rows, len(dims)).astype(np.uint32)
    qm = np.repeat(np.arange(len(dims)), len(rows)).astype(np.uint32)
    out = db.distances_ids(qs, ids, qm, 1)
    dec = oracle.sq8_decode(codes[rows], mins, scale)  # (rows, d)
    want = -dec[:, dims].T.reshape(-1)
    assert np.array_equal(out.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_bfs_matches_oracle_trace(gpu, oracle):
    """Lock-step BFS (DiskProvider::search_batch) through the GPU id-gather path reproduces the oracle
    trace on the committed 2,000-node graph (fp32 and SQ8)."""
    z = np.load(GOLD / "bfs_2k.npz")
    a = mt19937_uniform(2000 * 32 + 20 * 32, seed=7)
    x, qs = a[: 2000 * 32].reshape(2000, 32), a[2000 * 32:].reshape(20, 32)
    db = gpu.DiskannDeviceDB(x, 0)
    ids, dists, st = db.search_batch(z["adj"], [0, 999], qs, 10, 48)
    assert (ids == z["ids"]).mean() >= 0.99   # FP order can change a trajectory
    assert np.allclose(dists[ids == z["ids"]], z["dists"][ids == z["ids"]], rtol=1e-5, atol=1e-6)
    assert abs(st["evals"] - z["stats"][0]) <= 0.01 * z["stats"][0]
    mins, scale = oracle.sq8_train(x)
    db8 = gpu.DiskannDeviceDB(oracle.sq8_encode(x, mins, scale), 1, mins, scale)
    ids8, _, _ = db8.search_batch(z["adj"], [0, 999], qs, 10, 48)
    assert (ids8 == z["ids_sq8"]).mean() >= 0.99


def test_bfs_sql_known_answers(gpu, oracle):
    case = SQL["diskann_batch"]
    xb = np.array(case["xb"], np.float32)
    n = len(xb)
    adj = np.array([[j for j in range(n) if j != i] for i in range(n)], np.uint32)
    qs = np.array([qc["q"] for qc in case["queries"]], np.float32)
    ids, dists, _ = gpu.DiskannDeviceDB(xb, 0).search_batch(adj, [0], qs, 2, 8)
    for i, qc in enumerate(case["queries"]):
        assert ids[i].tolist() == qc["ids"] and np.allclose(dists[i], qc["dists"])
    sq = SQL["diskann_sq8_top1"]
    xb = np.array(sq["xb"], np.float32)
    n = len(xb)
    adj = np.array([[j for j in range(n) if j != i] for i in range(n)], np.uint32)
    mins, scale = oracle.sq8_train(xb)
    db = gpu.DiskannDeviceDB(oracle.sq8_encode(xb, mins, scale), 1, mins, scale)
    ids, _, _ = db.search_batch(adj, [0], np.array([qc["q"] for qc in sq["queries"]], np.float32), 3, 8)
    assert [r[0] for r in ids.tolist()] == [qc["top1"] for qc in sq["queries"]]


def test_bfs_from_diskann_file(gpu, oracle, tmp_path):
    """.diskann v2 file with an SQ8 trailer → HBM DB → BFS (the C4 path end to end on a small graph)."""
    import diskann_format as F
    a = mt19937_uniform(3000 * 16 + 10 * 16, seed=3)
    x, qs = a[: 3000 * 16].reshape(3000, 16), a[3000 * 16:].reshape(10, 16)
    _, nn = oracle.flat_search(x, x, 13, 0)
    adj = nn[:, 1:].astype(np.uint32)
    mins, scale = oracle.sq8_train(x)
    codes = oracle.sq8_encode(x, mins, scale)
    p = tmp_path / "g.diskann"
    F.write_index(p, x, adj, [5], sq8=(mins, scale, codes))
    f = F.open_index(p)
    db = gpu.DiskannDeviceDB(f.sq8_codes, 1, f.sq8_min, f.sq8_scale)
    ids, dists, st = db.search_batch(f.adjacency, f.entry_points, qs, 10, 40)
    oi, od, ost = oracle.diskann_search_batch(f.adjacency, f.entry_points, qs, 10, 40, codes=f.sq8_codes,
                                              mins=f.sq8_min, scale=f.sq8_scale)
    assert (ids == oi).mean() >= 0.99


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("fmt", [0, 1])
def test_bfs_many_queries_parallel_host(gpu, oracle, metric, fmt):
    """nq = 600 spreads the host BFS phases over worker threads (fixed per-query slot layout); a ragged
    graph (u32::MAX padding after a varying degree, out-of-range ids, duplicate neighbours) and
    duplicate entry points exercise the visited/skip rules of disk_provider.rs:556-577."""
    rng = np.random.default_rng(11)
    n, d, R = 4000, 48, 24
    x = rng.standard_normal((n, d)).astype(np.float32)
    qs = (x[rng.integers(0, n, 600)] + 0.1 * rng.standard_normal((600, d))).astype(np.float32)
    _, nn = oracle.flat_search(x, x, R - 4 + 1, 0)
    adj = np.full((n, R), 0xFFFFFFFF, np.uint32)
    adj[:, : R - 4] = nn[:, 1:]
    adj[:, R - 4: R - 2] = rng.integers(0, n, (n, 2))
    adj[::7, R - 2] = n + 5          # out of range: skipped, not a sentinel
    adj[::5, 3] = adj[::5, 2]        # duplicate neighbour
    deg = rng.integers(R // 2, R + 1, n)
    adj[np.arange(R)[None, :] >= deg[:, None]] = 0xFFFFFFFF
    eps = [17, 17, 2500]
    if fmt == 0:
        db = gpu.DiskannDeviceDB(x, 0)
        kw = dict(vecs=x)
    else:
        mins, scale = oracle.sq8_train(x)
        codes = oracle.sq8_encode(x, mins, scale)
        db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
        kw = dict(codes=codes, mins=mins, scale=scale)
    ids, dists, st = db.search_batch(adj, eps, qs, 10, 40, metric)
    oi, od, ost = oracle.diskann_search_batch(adj, eps, qs, 10, 40, metric, **kw)
    assert (ids == oi).mean() >= 0.99
    same = ids == oi
    assert np.allclose(dists[same], od[same], rtol=1e-5, atol=1e-5)
    assert abs(st["evals"] - ost["evals"]) <= 0.01 * ost["evals"]
    assert abs(st["steps"] - ost["steps"]) <= 2
    # every row sorted ascending (insert_result keeps the list ordered)
    assert np.all(np.diff(dists, axis=1) >= 0)


def _ragged_graph(oracle, x, R, rng, extra_random=2):
    n = len(x)
    _, nn = oracle.flat_search(x, x, R - extra_random - 2 + 1, 0)
    adj = np.full((n, R), 0xFFFFFFFF, np.uint32)
    adj[:, : R - extra_random - 2] = nn[:, 1:]
    adj[:, R - extra_random - 2: R - 2] = rng.integers(0, n, (n, extra_random))
    adj[::7, R - 2] = n + 5          # out of range: skipped, not a sentinel
    adj[::5, 3] = adj[::5, 2]        # duplicate neighbour
    deg = rng.integers(R // 2, R + 1, n)
    adj[np.arange(R)[None, :] >= deg[:, None]] = 0xFFFFFFFF
    return adj


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("L", [40, 128, 200])
def test_resident_bfs_matches_oracle(gpu, oracle, metric, fmt, L):
    """GPU-resident traversal (one wavefront per query) vs the DiskProvider::search_batch restatement on
    a ragged graph (sentinel padding, out-of-range ids, duplicate neighbours, duplicate entry points)."""
    rng = np.random.default_rng(5)
    n, d, R = 5000, 64, 32
    x = rng.standard_normal((n, d)).astype(np.float32)
    qs = (x[rng.integers(0, n, 300)] + 0.1 * rng.standard_normal((300, d))).astype(np.float32)
    adj = _ragged_graph(oracle, x, R, rng)
    eps = [17, 17, 2500, n + 3]
    if fmt == 0:
        db = gpu.DiskannDeviceDB(x, 0)
        kw = dict(vecs=x)
    else:
        mins, scale = oracle.sq8_train(x)
        codes = oracle.sq8_encode(x, mins, scale)
        db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
        kw = dict(codes=codes, mins=mins, scale=scale)
    db.register_graph(adj)
    ids, dists, st = db.search_batch_resident(eps, qs, 10, L, metric)
    assert st["pops"] > 0 and st["host_requeries"] == 0
    oi, od, ost = oracle.diskann_search_batch(adj, eps, qs, 10, L, metric, **kw)
    assert (ids == oi).mean() >= 0.99
    same = ids == oi
    assert np.allclose(dists[same], od[same], rtol=1e-5, atol=1e-4)
    assert abs(st["evals"] - ost["evals"]) <= 0.01 * ost["evals"]
    assert abs(st["steps"] - ost["steps"]) <= 2
    assert np.all(np.diff(dists, axis=1) >= 0)


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("L", [8, 24, 64])
def test_resident_bfs_exact_ties(gpu, oracle, fmt, L):
    """Small-integer data: every distance is exact in fp32 on both sides, and duplicated rows make exact
    ties everywhere (the result-list binary search, boundary evictions, the spill list).  The GPU
    traversal must then reproduce the oracle's ids, distances, evaluation count and step count exactly."""
    rng = np.random.default_rng(9)
    n, d, R = 3000, 16, 24
    base = rng.integers(0, 4, (n // 4, d)).astype(np.float32)
    x = np.repeat(base, 4, axis=0)[rng.permutation(n)]          # every row 4x
    x[0, :] = 0.0
    x[1, :] = 255.0                                              # SQ8: min 0, scale 255 → code == value
    if fmt == 1:
        x[2:] = np.clip(x[2:], 0, 3)
    qs = rng.integers(0, 4, (200, d)).astype(np.float32)
    adj = _ragged_graph(oracle, x, R, rng, extra_random=4)
    if fmt == 0:
        db = gpu.DiskannDeviceDB(x, 0)
        kw = dict(vecs=x)
    else:
        mins, scale = oracle.sq8_train(x)
        assert np.all(mins == 0) and np.all(scale == 255)
        codes = oracle.sq8_encode(x, mins, scale)
        db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
        kw = dict(codes=codes, mins=mins, scale=scale)
    db.register_graph(adj)
    ids, dists, st = db.search_batch_resident([0, 7], qs, 10, L)
    oi, od, ost = oracle.diskann_search_batch(adj, [0, 7], qs, 10, L, 0, **kw)
    assert np.array_equal(ids, oi)
    assert np.array_equal(dists, od)
    assert st["evals"] == ost["evals"]
    assert st["steps"] == ost["steps"]


def test_resident_bfs_host_fallback_shapes(gpu, oracle):
    """Shapes outside the kernel (R > 64) run through the host BFS with identical semantics."""
    rng = np.random.default_rng(2)
    n, d, R = 1500, 32, 80
    x = rng.standard_normal((n, d)).astype(np.float32)
    qs = x[:50] + 0.05
    adj = _ragged_graph(oracle, x, R, rng)
    db = gpu.DiskannDeviceDB(x, 0)
    db.register_graph(adj)
    ids, dists, st = db.search_batch_resident([3], qs, 10, 32)
    assert st["pops"] == 0 and st["host_requeries"] == 50
    hi, hd, _ = db.search_batch(adj, [3], qs, 10, 32)
    assert np.array_equal(ids, hi)


def test_resident_bfs_sql_known_answers(gpu, oracle):
    case = SQL["diskann_batch"]
    xb = np.array(case["xb"], np.float32)
    n = len(xb)
    adj = np.array([[j for j in range(n) if j != i] for i in range(n)], np.uint32)
    qs = np.array([qc["q"] for qc in case["queries"]], np.float32)
    db = gpu.DiskannDeviceDB(xb, 0)
    db.register_graph(adj)
    ids, dists, _ = db.search_batch_resident([0], qs, 2, 8)
    for i, qc in enumerate(case["queries"]):
        assert ids[i].tolist() == qc["ids"] and np.allclose(dists[i], qc["dists"])
