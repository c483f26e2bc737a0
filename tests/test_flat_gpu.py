"""GPU parity tests of the Flat path (libhipann.so) against the oracle (FAISS IndexFlat restatement).

Mirrors faiss-metal/tests/test_metal_flat.mm (same shapes, same std::mt19937(42) inputs, k up to 128)
but with a stricter pass rule than the reference's "top-1 exact" (test_metal_flat.mm:24-60): full
id/order parity except inside near-tie windows (tests/_data.py check_topk_parity).
"""
from __future__ import annotations

import json
import sys
import threading
from pathlib import Path

import numpy as np
import pytest

from _data import check_topk_parity, faiss_metal_case, mt19937_uniform

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
SQL = json.loads((GOLD / "sql_known_answers.json").read_text())
sys.path.insert(0, str(GOLD))
from make_golden import FLAT_CASES  # noqa: E402


@pytest.mark.parametrize("nv,nq,d,k,metric", FLAT_CASES)
def test_flat_faiss_metal_shapes(gpu, oracle, nv, nq, d, k, metric):
    xb, xq = faiss_metal_case(nv, nq, d)
    ix = gpu.HipIndexFlat(d, metric, xb)
    D, I = ix.search(xq, k)
    z = np.load(GOLD / "flat_mt19937.npz")
    key = f"flat_{nv}_{nq}_{d}_{k}_{metric}"
    Io, Do = z[key + "_I"].astype(np.int64), z[key + "_D"]
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    assert (I[:, 0] == Io[:, 0]).all(), "top-1 must match exactly (test_metal_flat.mm:51-59)"


@pytest.mark.parametrize("name", [k for k in SQL if k.startswith(("faiss_basic", "edge_"))])
def test_flat_sql_known_answers(gpu, name):
    case = SQL[name]
    xb = np.array(case["xb"], np.float32)
    deleted = set(case.get("deleted", []))
    ix = gpu.HipIndexFlat(xb.shape[1], case["metric"], xb)
    for qc in case["queries"]:
        k = qc["k"]
        req = min(k + len(deleted), len(xb))  # FaissIndex::Search (src/faiss_index.cpp:713-716)
        D, I = ix.search(np.array([qc["q"]], np.float32), req)
        keep = [(d, i) for d, i in zip(D[0], I[0]) if i >= 0 and i not in deleted][:k]
        ids = [int(i) for _, i in keep]
        dists = [float(d) for d, _ in keep]
        if "ids" in qc:
            assert ids == qc["ids"], (ids, qc)
        if "dists" in qc:
            assert np.allclose(dists, qc["dists"], rtol=2.5e-7, atol=1e-9), (dists, qc["dists"])
        if "n_below_0.01" in qc:
            assert sum(d < 0.01 for d in dists) == qc["n_below_0.01"]
        if "n_results" in qc:
            assert len(ids) == qc["n_results"]


@pytest.mark.parametrize("nq", [1, 19, 20, 21, 127, 128, 129, 300])
@pytest.mark.parametrize("metric", [0, 1])
def test_flat_batch_sizes_across_blas_threshold(gpu, oracle, nq, metric):
    xb, xq = faiss_metal_case(4000, nq, 64)
    ix = gpu.HipIndexFlat(64, metric, xb)
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)


@pytest.mark.parametrize("d,nq", [(1536, 11), (1536, 17), (1536, 19), (2048, 9), (4096, 5), (16384, 2)])
@pytest.mark.parametrize("n", [700, 5000])
def test_flat_small_batch_large_dimension(gpu, oracle, d, nq, n):
    """nq < 20 (FAISS's non-BLAS path) with d·nq beyond the direct scan's 64 KiB of queries in LDS: the batch runs as
    query chunks (before r06 this raised "dimension too large for the scan path", also for an IVF coarse step)."""
    xb, xq = faiss_metal_case(n, nq, d)
    for metric in (0, 1):
        ix = gpu.HipIndexFlat(d, metric, xb)
        D, I = ix.search(xq, 7)
        Do, Io = oracle.flat_search(xb, xq, 7, metric)
        check_topk_parity(xb, xq, D, I, Do, Io, metric)


@pytest.mark.parametrize("d", [1, 3, 5, 31, 33, 100, 130, 2048])
def test_flat_odd_dimensions(gpu, oracle, d):
    xb, xq = faiss_metal_case(700, 24, d)
    for nq in (3, 24):
        ix = gpu.HipIndexFlat(d, 0, xb)
        D, I = ix.search(xq[:nq], 7)
        Do, Io = oracle.flat_search(xb, xq[:nq], 7)
        check_topk_parity(xb, xq[:nq], D, I, Do, Io, 0, min_exact=0.97 if d <= 3 else 0.99)


@pytest.mark.parametrize("k", [1, 63, 64, 65, 200, 1000, 2048])
def test_flat_k_range(gpu, oracle, k):
    xb, xq = faiss_metal_case(5000, 22, 32)
    for nq in (4, 22):
        ix = gpu.HipIndexFlat(32, 0, xb)
        D, I = ix.search(xq[:nq], k)
        Do, Io = oracle.flat_search(xb, xq[:nq], k)
        check_topk_parity(xb, xq[:nq], D, I, Do, Io, 0, min_exact=0.98)


def test_flat_k_greater_than_ntotal_pads(gpu):
    xb = np.array([[1, 0, 0], [0, 1, 0]], np.float32)
    for metric, pad in ((0, np.inf), (1, -np.inf)):
        ix = gpu.HipIndexFlat(3, metric, xb)
        for nq in (1, 25):
            D, I = ix.search(np.tile(np.array([[1, 0, 0]], np.float32), (nq, 1)), 100)
            assert I.shape == (nq, 100)
            assert (I[:, :2] == [0, 1]).all() and (I[:, 2:] == -1).all()
            assert (D[:, 2:] == pad).all()   # MetalIndexFlat.mm:355-368 sentinels


def test_flat_empty_index_and_batch(gpu):
    ix = gpu.HipIndexFlat(8, 0)
    D, I = ix.search(np.zeros((3, 8), np.float32), 4)
    assert (I == -1).all() and np.isinf(D).all() and (D > 0).all()
    D, I = ix.search(np.zeros((0, 8), np.float32), 4)
    assert D.shape == (0, 4)
    ix.add(np.eye(8, dtype=np.float32))
    with pytest.raises(gpu.HipAnnError):
        ix.search(np.zeros((1, 8), np.float32), 0)      # k <= 0 throws (MetalIndexFlat.mm:297)
    with pytest.raises(gpu.HipAnnError):
        ix.search(np.zeros((1, 8), np.float32), gpu.MAX_K + 1)
    with pytest.raises(ValueError):
        ix.search(np.zeros((1, 7), np.float32), 1)


def test_flat_incremental_add_and_reconstruct(gpu, oracle):
    xb, xq = faiss_metal_case(3000, 30, 40)
    ix = gpu.HipIndexFlat(40, 0)
    for s in range(0, 3000, 700):
        ix.add(xb[s:s + 700])
    assert ix.ntotal == 3000
    assert np.array_equal(ix.reconstruct(1234), xb[1234])
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10)
    check_topk_parity(xb, xq, D, I, Do, Io)


def test_flat_ties_order_by_label(gpu):
    # 300 identical rows: every distance ties; FAISS returns the lowest labels in label order
    xb = np.tile(np.array([[0.5, -0.25, 1.0, 0.0]], np.float32), (300, 1))
    ix = gpu.HipIndexFlat(4, 0, xb)
    for nq in (1, 40):
        D, I = ix.search(np.zeros((nq, 4), np.float32), 37)
        assert (I == np.arange(37)).all()


def test_flat_multi_shard_same_device(gpu, oracle):
    """Rows sharded over devices [0, 0] (two shards on one GPU) → peer gather + device merge."""
    xb, xq = faiss_metal_case(5001, 30, 64)
    ix = gpu.HipIndexFlat(64, 0, xb, devices=[0, 0])
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10)
    check_topk_parity(xb, xq, D, I, Do, Io)
    D1, I1 = ix.search(xq[:5], 10)
    check_topk_parity(xb, xq[:5], D1, I1, Do[:5], Io[:5])


def test_flat_device_api_and_merge(gpu, oracle):
    import torch
    xb, xq = faiss_metal_case(6000, 64, 96)
    dev = torch.device("cuda", 0)
    xb_t = torch.from_numpy(xb).to(dev)
    xq_t = torch.from_numpy(xq).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    parts_D, parts_I = [], []
    for lo, hi in ((0, 2500), (2500, 6000)):   # two "ranks"
        sh = gpu.HipIndexFlatDevice(96, 0, xb_t[lo:hi].data_ptr(), hi - lo, 0, copy=False, label_offset=lo)
        Dp = torch.empty((64, 10), device=dev)
        Ip = torch.empty((64, 10), device=dev, dtype=torch.int64)
        sh.search_device(64, xq_t.data_ptr(), 10, Dp.data_ptr(), Ip.data_ptr(), stream)
        torch.cuda.synchronize()
        parts_D.append(Dp)
        parts_I.append(Ip)
        sh.close()
    Da, Ia = torch.stack(parts_D).contiguous(), torch.stack(parts_I).contiguous()
    D = torch.empty((64, 10), device=dev)
    I = torch.empty((64, 10), device=dev, dtype=torch.int64)
    gpu.merge_topk_device(0, 2, 64, 10, Da.data_ptr(), Ia.data_ptr(), D.data_ptr(), I.data_ptr(), stream)
    torch.cuda.synchronize()
    Do, Io = oracle.flat_search(xb, xq, 10)
    check_topk_parity(xb, xq, D.cpu().numpy(), I.cpu().numpy(), Do, Io)


def test_merge_kernel_lexicographic(gpu):
    """merge_topk_device = k smallest (key, label) of the union; pads (-1) ignored; IP descending."""
    import torch
    rng = np.random.default_rng(3)
    for metric in (0, 1):
        P, nq, k = 5, 33, 17
        D = rng.integers(0, 6, (P, nq, k)).astype(np.float32)  # many exact ties
        I = rng.permutation(P * nq * k).reshape(P, nq, k).astype(np.int64)
        I[rng.random((P, nq, k)) < 0.1] = -1
        dev = torch.device("cuda", 0)
        Dt, It = torch.from_numpy(D).to(dev), torch.from_numpy(I).to(dev)
        Do = torch.empty((nq, k), device=dev)
        Io = torch.empty((nq, k), device=dev, dtype=torch.int64)
        gpu.merge_topk_device(metric, P, nq, k, Dt.data_ptr(), It.data_ptr(), Do.data_ptr(), Io.data_ptr(), 0)
        torch.cuda.synchronize()
        Do, Io = Do.cpu().numpy(), Io.cpu().numpy()
        for q in range(nq):
            c = sorted(((D[p, q, j] if metric == 0 else -D[p, q, j]), I[p, q, j])
                       for p in range(P) for j in range(k) if I[p, q, j] >= 0)[:k]
            assert Io[q].tolist() == [lab for _, lab in c] + [-1] * (k - len(c))


def test_flat_concurrent_searches_one_handle(gpu, oracle):
    xb, xq = faiss_metal_case(3000, 50, 64)
    ix = gpu.HipIndexFlat(64, 0, xb)
    ref = ix.search(xq, 10)
    out = [None] * 8

    def run(t):
        out[t] = ix.search(xq, 10)

    ts = [threading.Thread(target=run, args=(t,)) for t in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for o in out:
        assert np.array_equal(o[1], ref[1]) and np.array_equal(o[0], ref[0])


def test_flat_backend_cpu_to_gpu(gpu, oracle):
    be = gpu.get_gpu_backend()
    assert be.is_available() and be.backend_name() == "hip" and "gfx950" in be.device_info()
    xb, xq = faiss_metal_case(1000, 10, 32)
    g = be.cpu_to_gpu({"type": "Flat", "d": 32, "metric": 0, "xb": xb})
    D, I = g.search(xq, 5)
    Do, Io = oracle.flat_search(xb, xq, 5)
    check_topk_parity(xb, xq, D, I, Do, Io)
    back = be.gpu_to_cpu(g)
    assert np.array_equal(back["xb"], xb)
    with pytest.raises(RuntimeError):
        be.cpu_to_gpu({"type": "HNSW"})


def test_flat_large_properties(gpu, oracle):
    """200k x 768, nq = 1024 (BLAS form): self-queries find themselves at ~0, the output is sorted, and a
    query subset matches the oracle."""
    import torch
    n, d, nq = 200_000, 768, 1024
    g = torch.Generator().manual_seed(5)
    xb = (torch.rand((n, d), generator=g) * 2 - 1).numpy()
    sel = np.arange(0, n, n // nq)[:nq]
    xq = xb[sel].copy()
    ix = gpu.HipIndexFlat(d, 0, xb)
    D, I = ix.search(xq, 10)
    assert (I[:, 0] == sel).all()
    assert (np.abs(D[:, 0]) < 1e-2).all()
    assert (np.diff(D, axis=1) >= 0).all()
    Do, Io = oracle.flat_search(xb, xq[:64], 10)  # oracle BLAS path on a 64-query subset
    check_topk_parity(xb, xq[:64], D[:64], I[:64], Do, Io)


@pytest.mark.parametrize("form", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("nq,d", [(20, 64), (129, 33), (300, 768), (64, 5), (257, 100), (600, 96)])
def test_flat_forms_blas_path(gpu, oracle, form, metric, nq, d):
    """hipann_flat_set_form: the fp32 (0), 3-term split-bf16 (1) and exact (3, default: 2-term filter +
    direct-form rerank) forms of the batched path meet the fp32 parity rule; the 2-term split (2,
    measurement only) keeps ≈2^-16 relative products, so only its recall is checked."""
    xb, xq = faiss_metal_case(20000, nq, d)  # > 16384 rows: the fused path (smaller tables select from keys)
    ix = gpu.HipIndexFlat(d, metric, xb)
    assert ix.form == ix.FORM_I8_EXACT
    ix.form = form
    assert ix.form == form
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    if form != 2:
        check_topk_parity(xb, xq, D, I, Do, Io, metric)
    else:
        hit = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(I.tolist(), Io.tolist())])
        assert hit >= 0.97, hit
    with pytest.raises(gpu.HipAnnError):
        ix.form = 6


def test_flat_exact_form_ties_fall_back(gpu, oracle):
    """Exact form with 40 copies of every row: the 16 kept scan candidates are all ties, the bound check
    cannot exclude a pruned copy, so every query re-runs on the 3-term path; results keep parity."""
    base, xq = faiss_metal_case(500, 64, 48)
    xb = np.repeat(base, 40, axis=0)  # 20000 rows: the fused path
    ix = gpu.HipIndexFlat(48, 0, xb)
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10, 0)
    check_topk_parity(xb, xq, D, I, Do, Io, 0)
    assert ix.rerank_fallbacks() == 64


def test_flat_exact_form_large_k_uses_split3(gpu, oracle):
    xb, xq = faiss_metal_case(20000, 40, 32)
    ix = gpu.HipIndexFlat(32, 1, xb)
    D, I = ix.search(xq, 50)   # k > 12: the 3-term path, no rerank
    Do, Io = oracle.flat_search(xb, xq, 50, 1)
    check_topk_parity(xb, xq, D, I, Do, Io, 1)
    assert ix.rerank_fallbacks() == 0


@pytest.mark.parametrize("form", [3, 4])
def test_flat_exact_form_matches_fp32_form_at_scale(gpu, form):
    """Large-size property: the exact form (2-term split filter + direct-form rerank) returns the fp32
    form's lists except inside near-tie windows (distances within the fp32 rounding scale), on
    200k × 128 with 512 queries."""
    rng = np.random.default_rng(7)
    xb = rng.standard_normal((200_000, 128), dtype=np.float32)
    xq = rng.standard_normal((512, 128), dtype=np.float32)
    ix = gpu.HipIndexFlat(128, 0, xb)
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    ix.form = form
    D1, I1 = ix.search(xq, 10)
    scale = np.sum(xq.astype(np.float64) ** 2, 1)[:, None] + np.max(np.sum(xb.astype(np.float64) ** 2, 1))
    assert (np.abs(D1 - D0) <= 1e-5 * scale).all()
    assert (I1 == I0).mean() >= 0.995


@pytest.mark.parametrize("form", [4, 5])
@pytest.mark.parametrize("metric", [0, 1])
def test_flat_bf16_two_pass_resume(gpu, oracle, metric, form):
    """The bf16 filter's two-pass schedule (1M rows, 64 splits of 61 tiles, nq = 512: pass A over the first
    6 tiles of every split under the 64K-row seed bound, the bound re-merged, pass B resumed from pass A's
    lists): the fp32 form's lists except inside near-tie windows, and the oracle's parity rule on a
    query subset."""
    rng = np.random.default_rng(11)
    n, d, nq = 1_000_000, 64, 512
    xb = rng.standard_normal((n, d), dtype=np.float32)
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    ix = gpu.HipIndexFlat(d, metric, xb)
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    ix.form = form
    D1, I1 = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == form
    scale = np.sum(xq.astype(np.float64) ** 2, 1)[:, None] + np.max(np.sum(xb.astype(np.float64) ** 2, 1))
    assert (np.abs(D1 - D0) <= 1e-5 * scale).all()
    assert (I1 == I0).mean() >= 0.995
    Do, Io = oracle.flat_search(xb, xq[:48], 10, metric)
    check_topk_parity(xb, xq[:48], D1[:48], I1[:48], Do, Io, metric)


@pytest.mark.parametrize("form", [4, 5])
@pytest.mark.parametrize("metric", [0, 1])
def test_flat_bf16_flagged_queries_candidate_rerank(gpu, oracle, metric, form):
    """Bounded passes with near-duplicate rows (16K base rows x 40 copies + 1e-4 noise, shuffled; 640K x 64,
    nq 256): every query's 32 best scan keys are copies of one base row, so the first rerank cannot certify
    it and flags it.  The second rerank recomputes all of a flagged query's buffered candidates and
    certifies against the pass bound (the 32nd best key of pass A's rows, several base rows away); only
    what it cannot certify re-runs on SPLIT3.  Ids follow the oracle's parity rule on every query.
    Reference edge case: duplicate vectors (test/sql/edge_cases.test:75-83)."""
    rng = np.random.default_rng(23 + metric)
    base = rng.standard_normal((16_000, 64), dtype=np.float32)
    xb = np.repeat(base, 40, axis=0)
    xb += 1e-4 * rng.standard_normal(xb.shape, dtype=np.float32)
    xb = xb[rng.permutation(len(xb))]
    xq = rng.standard_normal((256, 64), dtype=np.float32)
    ix = gpu.HipIndexFlat(64, metric, xb)
    assert ix.form == ix.FORM_I8_EXACT
    ix.form = form
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == form
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    # the first rerank flags nearly all of these queries; the candidate rerank certifies most of them
    assert ix.rerank_fallbacks() < len(xq) // 4, ix.rerank_fallbacks()


@pytest.mark.parametrize("n", [200, 1000, 3000])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [1, 7, 32, 64])
def test_flat_small_table_select_exact_ties(gpu, oracle, n, metric, k):
    """Small tables at nq >= 20 (the IVF coarse quantizer's shape): GEMM keys + one select per key row
    (the bitwise select for <= 1024 columns, the list path beyond).  Small-integer data makes every
    product exact, so keys tie exactly and the (distance, label) order alone decides: ids and distances
    must equal the oracle's bit for bit, including an all-zero query (IP keys +-0 for every row)."""
    rng = np.random.default_rng(n * 10 + k + metric)
    d = 24
    xb = rng.integers(-2, 3, size=(n, d)).astype(np.float32)
    xq = rng.integers(-2, 3, size=(40, d)).astype(np.float32)
    xq[5] = 0.0
    ix = gpu.HipIndexFlat(d, metric, xb)
    D, I = ix.search(xq, k)
    Do, Io = oracle.flat_search(xb, xq, k, metric)
    assert np.array_equal(I, Io)
    assert np.array_equal(D, Do)


def test_flat_ip_four_shards_in_process_c5_path(gpu, oracle):
    """The extension's in-process multi-device handle (hipann_flat_create with devices [0, 0, 0, 0]): rows
    sharded contiguously over four shards, each shard searched with its own stream and scratch (the bounded-pass
    bf16 filter: 1M rows per shard), per-shard top-k gathered by peer copy onto shard 0's device and merged
    (DESIGN §7).  C5's per-GPU path (Flat IP, d 768, batch 1024) at 1M rows per shard: ids equal a single-shard
    index's exact fp32 form except in near-tie windows, and follow the oracle's parity rule on 12 queries."""
    rng = np.random.default_rng(55)
    n, d, nq = 4_000_000, 768, 1024
    xb = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    ix4 = gpu.HipIndexFlat(d, 1, xb, devices=[0, 0, 0, 0])
    D4, I4 = ix4.search(xq, 10)
    assert ix4.rerank_fallbacks() == 0
    ix4.close()
    ix1 = gpu.HipIndexFlat(d, 1, xb)
    ix1.form = ix1.FORM_FP32
    D1, I1 = ix1.search(xq, 10)
    ix1.close()
    assert (I4 == I1).mean() >= 0.995
    scale = np.sqrt(np.sum(xq.astype(np.float64) ** 2, 1))[:, None] * np.sqrt(d)
    assert (np.abs(D4 - D1) <= 1e-5 * scale).all()
    Do, Io = oracle.flat_search(xb, xq[:12], 10, 1)
    check_topk_parity(xb, xq[:12], D4[:12], I4[:12], Do, Io, 1)


@pytest.mark.parametrize("metric", [0, 1])
def test_flat_i8_form_row_scales_and_edge_rows(gpu, oracle, metric):
    """Form 5 (int8 filter): per-row scales over rows whose magnitudes span 2^-20 .. 2^20 (the scale follows each
    row, the bound follows the measured residuals), all-zero rows and an all-zero query, a query equal to a row;
    600k x 128, nq 256, the oracle's parity rule on 40 queries and the fp32 form's ids elsewhere."""
    rng = np.random.default_rng(91 + metric)
    n, d, nq = 600_000, 128, 256
    xb = rng.standard_normal((n, d), dtype=np.float32)
    xb *= np.exp2(rng.integers(-20, 21, size=(n, 1))).astype(np.float32)
    xb[::1000] = 0.0
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    xq[7] = 0.0
    xq[8] = xb[12345]
    ix = gpu.HipIndexFlat(d, metric, xb)
    ix.form = ix.FORM_I8_EXACT
    D, I = ix.search(xq, 10)
    assert ix.last_search_path() == {"form": 5, "filter_k": 64, "sublists": 0}
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    assert (I == I0).mean() >= 0.99
    Do, Io = oracle.flat_search(xb, xq[:40], 10, metric)
    check_topk_parity(xb, xq[:40], D[:40], I[:40], Do, Io, metric)
    if metric == 0:
        assert I[8, 0] == 12345 and D[8, 0] == 0.0
    ix.close()


@pytest.mark.parametrize("nq", [4096, 8192])
def test_flat_bf16_large_batch_buffers_do_not_overflow(gpu, oracle, nq):
    """Large batches on the bounded passes: the per-(query, split) candidate buffer is sized from
    the expected fill (k · rows / sample over the splits), so at nq 4096 and 8192 (few splits per query block,
    many rows per split) no query overflows into the SPLIT3 re-run.  2M x 128 uniform rows: ids equal the fp32
    form's except in near-tie windows, re-runs stay under 1% of the batch, and the oracle's parity rule holds on
    16 queries."""
    rng = np.random.default_rng(nq)
    n, d = 2_000_000, 128
    xb = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    ix = gpu.HipIndexFlat(d, 0, xb)
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == ix.FORM_I8_EXACT
    assert ix.rerank_fallbacks() <= nq // 100, ix.rerank_fallbacks()
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    assert (I == I0).mean() >= 0.995
    scale = np.sum(xq.astype(np.float64) ** 2, 1)[:, None] + np.max(np.sum(xb.astype(np.float64) ** 2, 1))
    assert (np.abs(D - D0) <= 1e-5 * scale).all()
    Do, Io = oracle.flat_search(xb, xq[:16], 10, 0)
    check_topk_parity(xb, xq[:16], D[:16], I[:16], Do, Io, 0)


@pytest.mark.parametrize("n,d,nq,expect", [(600_000, 1280, 256, 4), (600_000, 128, 200, 4), (300_000, 128, 256, 4),
                                           (600_000, 1024, 256, 5)])
def test_flat_default_form_falls_back_where_int8_does_not_run(gpu, oracle, n, d, nq, expect):
    """The default form 5 runs only as the bounded passes with d <= 1024 (exact int32 sums), nq >= 256 and
    >= 512K rows; other shapes run form 4 (the bf16 image), and the path reports the form that ran.  Ids follow
    the oracle's parity rule on 16 queries either way."""
    rng = np.random.default_rng(n + d + nq)
    xb = rng.standard_normal((n, d), dtype=np.float32)
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    ix = gpu.HipIndexFlat(d, 0, xb)
    assert ix.form == ix.FORM_I8_EXACT
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == expect, ix.last_search_path()
    Do, Io = oracle.flat_search(xb, xq[:16], 10, 0)
    check_topk_parity(xb, xq[:16], D[:16], I[:16], Do, Io, 0)
    assert ix.rerank_fallbacks() == 0
    ix.close()


@pytest.mark.parametrize("scaled", [False, True])
@pytest.mark.parametrize("nq", [1, 3, 16, 17])
@pytest.mark.parametrize("metric", [0, 1])
def test_flat_small_batch_int8_filter(gpu, oracle, nq, metric, scaled):
    """nq < 20 (FAISS's direct-form path, the extension's per-query call) on a large table: the int8 image as the
    filter (flat_i8_scan, 64 candidates per query) and the exact direct-form rerank — ids and distances follow the
    oracle's direct-form parity rule, few query re-runs; 17+ queries and HIPANN_FLAT_I8_SMALL=0 take the fp32 scan.
    Includes a query equal to a row (distance 0); `scaled`: rows with magnitudes over 2^-10 .. 2^10, whose largest
    int8 residual makes the bound too loose to certify — every query re-runs on the fp32 scan, same results."""
    rng = np.random.default_rng(7 * nq + metric)
    n, d = 300_000, 192
    xb = rng.standard_normal((n, d), dtype=np.float32)
    if scaled:
        xb *= np.exp2(rng.integers(-10, 11, size=(n, 1))).astype(np.float32)
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    xq[0] = xb[4321]
    ix = gpu.HipIndexFlat(d, metric, xb)
    D, I = ix.search(xq, 10)
    path = ix.last_search_path()
    assert path["form"] == (ix.FORM_I8_EXACT if nq <= 16 else ix.FORM_FP32), path
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    if metric == 0:
        assert I[0, 0] == 4321 and D[0, 0] == 0.0
    if not scaled:  # the bound is conservative: a query whose 10th distance sits near its 64th key re-runs
        assert ix.rerank_fallbacks() <= max(1, nq // 4), ix.rerank_fallbacks()
    ix.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_flat_multi_shard_concurrent_one_host_sync(gpu, oracle, metric):
    """the in-process multi-device handle (devices [0, 0, 0, 0]) launches every shard before it waits
    on any — one host synchronisation per hipann_flat_search once the images exist, which also reads every shard's
    exact-form flag count — on the batched int8 bounded passes (nq 256, 600K rows per shard) and the small-batch
    int8 scan (nq 4); ids follow the oracle's parity rule."""
    rng = np.random.default_rng(77 + metric)
    n, d = 2_400_000, 128
    xb = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    xq = rng.uniform(-1, 1, (256, d)).astype(np.float32)
    ix = gpu.HipIndexFlat(d, metric, xb, devices=[0, 0, 0, 0])
    for nq in (256, 4):
        ix.search(xq[:nq], 10)  # builds the images (their own syncs)
        s0 = ix.host_syncs()
        for _ in range(3):
            D, I = ix.search(xq[:nq], 10)
        assert ix.host_syncs() - s0 == 3, (nq, ix.host_syncs() - s0)
        assert ix.last_search_path()["form"] == ix.FORM_I8_EXACT
        Do, Io = oracle.flat_search(xb, xq[:nq][:32], 10, metric)
        check_topk_parity(xb, xq[:nq][:32], D[:32], I[:32], Do, Io, metric)
    assert ix.rerank_fallbacks() == 0
    ix.close()


@pytest.mark.parametrize("nq", [256, 8])
def test_flat_multi_shard_flagged_queries_finish(gpu, oracle, nq):
    """Deferred completion with flagged queries: near-duplicate rows (the candidate-rerank case) over 4 shards on
    one device; the flagged shards re-run after the single synchronisation and the results are delivered again.
    Ids follow the oracle's parity rule on every query."""
    rng = np.random.default_rng(31 + nq)
    base = rng.standard_normal((4_000, 64), dtype=np.float32)
    xb = np.repeat(base, 80, axis=0)  # 80 copies: deeper than any filter (64), so the bound check flags
    xb += 1e-4 * rng.standard_normal(xb.shape, dtype=np.float32)
    xb = xb[rng.permutation(len(xb))]
    xq = rng.standard_normal((nq, 64), dtype=np.float32)
    ix = gpu.HipIndexFlat(64, 0, xb, devices=[0, 0, 0, 0])
    D, I = ix.search(xq, 10)
    assert ix.rerank_fallbacks() > 0  # the deferred re-runs ran
    Do, Io = oracle.flat_search(xb, xq, 10)
    check_topk_parity(xb, xq, D, I, Do, Io)
    ix.close()


@pytest.mark.parametrize("metric", [0, 1])
def test_flat_successive_appends_incremental(gpu, oracle, metric):
    """20 successive 2048-row appends after the int8 and bf16 images exist.  Each append tiles
    only the tiles holding new rows and updates max ‖x‖² and the residual maxima as running maxima; the batched int8
    passes (nq 256), the bf16 passes (form 4) and the small-batch int8 scan (nq 4) on the grown table follow the
    oracle's parity rule, and the last chunk (rows ×3) is found by the queries placed next to it."""
    rng = np.random.default_rng(61 + metric)
    d, n0, step, steps = 64, 600_000, 2048, 20
    xb = rng.uniform(-1, 1, (n0 + step * steps, d)).astype(np.float32)
    xb[-step:] *= np.float32(3.0)
    xq = rng.uniform(-1, 1, (256, d)).astype(np.float32)
    xq[:16] = xb[-16:] + np.float32(1e-3)
    ix = gpu.HipIndexFlat(d, metric, xb[:n0])
    ix.search(xq, 10)          # int8 image (bounded passes)
    ix.form = ix.FORM_BF16_EXACT
    ix.search(xq, 10)          # bf16 image
    ix.form = ix.FORM_I8_EXACT
    ix.search(xq[:4], 10)      # small-batch int8 scan
    for a in range(steps):
        lo = n0 + a * step
        ix.add(xb[lo:lo + step])
    assert ix.ntotal == len(xb)
    Do, Io = oracle.flat_search(xb, xq[:64], 10, metric)
    for form, nq in ((ix.FORM_I8_EXACT, 256), (ix.FORM_BF16_EXACT, 256), (ix.FORM_I8_EXACT, 4)):
        ix.form = form
        D, I = ix.search(xq[:nq], 10)
        assert ix.last_search_path()["form"] == form, (form, nq)
        m = min(nq, 64)
        check_topk_parity(xb, xq[:m], D[:m], I[:m], Do[:m], Io[:m], metric)
        # a table built from scratch over the same rows: same answers, and the same bound terms (the running maxima
        # equal the rebuild's), so the same number of flagged re-runs
        fresh = gpu.HipIndexFlat(d, metric, xb)
        fresh.form = form
        before = ix.rerank_fallbacks()
        D2, I2 = fresh.search(xq[:nq], 10)
        D, I = ix.search(xq[:nq], 10)
        assert np.array_equal(I, I2) and np.array_equal(D, D2), (form, nq)
        assert ix.rerank_fallbacks() - before == fresh.rerank_fallbacks(), (form, nq)
        fresh.close()


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("nq", [4, 256])
def test_flat_nan_and_overflow_queries_pad_like_faiss(gpu, oracle, metric, nq):
    """a NaN query (and, for L2, a query whose distances overflow to +inf) is never admitted by FAISS's
    heap (strict C::cmp(top, dis) with NaN / inf against ±FLT_MAX), so the CPU path returns all −1 labels for it.
    The small-batch int8 scan (nq 4) and the int8 bounded passes (nq 256) return the same −1 labels, and the other
    queries of the batch keep the oracle's parity."""
    rng = np.random.default_rng(3 + metric)
    n, d = 600_000, 64
    xb = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
    xq[1, 5] = np.nan
    bad = [1]
    if metric == 0:
        xq[2] = np.float32(3e38)  # ‖q − x‖² overflows to +inf for every row
        bad.append(2)
    ix = gpu.HipIndexFlat(d, metric, xb)
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    for b in bad:
        assert (Io[b] == -1).all()
        assert (I[b] == -1).all(), (b, I[b])
    good = np.array([i for i in range(nq) if i not in bad])
    check_topk_parity(xb, xq[good], D[good], I[good], Do[good], Io[good], metric)
