"""GPU parity at the BASELINE configurations' shapes, against the oracle.

The benchmark configurations themselves (10M rows) are far beyond what the oracle finishes in seconds, so
each test runs the same code path at the largest shape the oracle checks quickly, with the same data
model, the same build (GPU k-means / k-NN graph / SQ8 codec) and the same batch:

* C1  Flat L2 10k × 128, k = 10 (the full C1 shape, the faiss-metal test inputs): the host-pointer C ABI
      (hipann_flat_search, the call the extension's FaissIndex::Search makes) at nq = 1 and nq = 1000;
      ids bit-identical to the oracle's CPU path (FAISS IndexFlatL2::search restatement).
* C2  Flat L2 1M × 768, nq = 1024, k = 10 (the full C2 shape): every form through the device API the
      bench uses; the oracle (FAISS BLAS-path restatement) on a 256-query subset.
* C3  IVFFlat nlist = 1024, nprobe = 32, d = 768, nq = 1024, k = 10 on 200k rows of the bench's
      low-rank data, built by ivf_build (the bench's GPU k-means + assignment): probe lists equal the
      oracle's (tie-tolerant) and ids follow the parity rule; forms 5 (default), 3 and 0.
* C4  DiskANN resident traversal at d = 1536 SQ8, R = 64, L = 128 on a 32k-node graph built by
      diskann_build (the bench's graph builder), plus the exact-tie integer variant (ids, distances,
      evaluation and step counts identical to the oracle).

Pattern: faiss-metal/tests/test_metal_ivfflat.mm:28-100 and test_metal_flat.mm:489-505 (GPU vs CPU FAISS
on the same data, top-k compared).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

from _data import TAU, check_probe_parity, check_topk_parity, oracle_on_gpu_probes

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
# identical probe lists given identical centroids.  Neither side's fp32 coarse keys are FAISS's own sgemm
# sums (the oracle's dot products are its compiler's SIMD order, the GPU's a 3-term bf16 split or fp32 MFMA tiles), so
# a centroid pair whose fp64 distances differ by less than the keys' rounding can swap at the nprobe boundary.  The
# rule held here: check_probe_parity asserts every differing rank is such a tie (fp64 gap <= 1e-6·(|q|² + max|c|²), the
# parity window; DESIGN §2 has the key error budget), at most C3_MAX_PROBE_DIFF of the 1024 queries differ
# (3 on the 200K-row C3 index, 0 on the 2M-row one, r06), and each such query's ids must equal the oracle's
# IndexIVF::search_preassigned over the GPU's own probe list — every query of the batch is checked.
C3_MAX_PROBE_DIFF = 5
sys.path.insert(0, str(ROOT))


def _dev_search(index, xq_t, k, torch):
    nq = xq_t.shape[0]
    D = torch.empty((nq, k), device=xq_t.device, dtype=torch.float32)
    I = torch.empty((nq, k), device=xq_t.device, dtype=torch.int64)
    index.search_device(nq, xq_t.data_ptr(), k, D.data_ptr(), I.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return D.cpu().numpy(), I.cpu().numpy()


@pytest.mark.parametrize("metric", [0, 1])
def test_c1_flat_10k_128(gpu, oracle, metric):
    """C1 (BASELINE configs[0]): 10k × 128, k = 10, at the extension's real call shape — FaissIndex::Search
    calls search(1, …) (src/faiss_index.cpp:737) — and as one 1000-query batch (SearchBatch, SURVEY §8f
    rank 1).  The CPU path the GPU must reproduce is FAISS's IndexFlatL2::search: the direct form at nq = 1,
    the BLAS form at nq = 1000.  nq = 1: ids identical to the oracle's, bit for bit (both direct form).
    nq = 1000: the BLAS form's dot products depend on the BLAS library's summation order (the oracle's
    restatement has its own, OpenBLAS another), so ids are identical except where two rows' fp64 distances
    lie within the parity rule's tie window (IP on this data: 1 query of 1000 at r03)."""
    from _data import faiss_metal_case

    xb, xq = faiss_metal_case(10_000, 1000, 128)
    ix = gpu.HipIndexFlat(128, metric, xb)
    # nq = 1: one call per query, as the per-query loops of ann_search.cpp:320-333 / :610-621 issue them
    D1 = np.empty((100, 10), np.float32)
    I1 = np.empty((100, 10), np.int64)
    for i in range(100):
        D1[i:i + 1], I1[i:i + 1] = ix.search(xq[i:i + 1], 10)
    Io1 = np.empty_like(I1)
    Do1 = np.empty_like(D1)
    for i in range(100):  # the oracle at nq = 1 (direct fvec_L2sqr / inner product form)
        Do1[i:i + 1], Io1[i:i + 1] = oracle.flat_search(xb, xq[i:i + 1], 10, metric)
    assert np.array_equal(I1, Io1), f"nq=1 ids differ on {(I1 != Io1).any(axis=1).sum()} queries"
    assert np.allclose(D1, Do1, rtol=2e-6, atol=1e-6)
    # nq = 1000: the BLAS-form path (FAISS: nq >= distance_compute_blas_threshold)
    D, I = ix.search(xq, 10)
    Do, Io = oracle.flat_search(xb, xq, 10, metric)
    st = check_topk_parity(xb, xq, D, I, Do, Io, metric)
    assert st["exact_fraction"] >= 0.999, st
    # a batch equals the loop of single-query calls (SearchBatch vs Search), up to the same
    # tie window (direct vs BLAS form)
    check_topk_parity(xb, xq[:100], D[:100], I[:100], D1, I1, metric)
    ix.close()


@pytest.fixture(scope="module")
def c2_data(gpu):
    import torch

    import bench

    dev = torch.device("cuda", 0)
    n, d, nq = 1_000_000, 768, 1024
    xb_t = torch.empty((n, d), device=dev, dtype=torch.float32)
    bench.gen_uniform_rows(torch, xb_t, 0, 42)  # the bench's C2 rows (U(-1,1), chunk-seeded)
    g = torch.Generator(device=dev).manual_seed(4242)
    xq_t = (torch.rand((nq, d), generator=g, device=dev) * 2 - 1).contiguous()
    torch.cuda.synchronize()
    return xb_t, xq_t, xb_t.cpu().numpy(), xq_t.cpu().numpy()


@pytest.fixture(scope="module")
def c2_oracle(c2_data, oracle):
    _, _, xb, xq = c2_data
    return oracle.flat_search(xb, xq, 10, 0)


@pytest.mark.parametrize("form", [5, 4, 3, 1, 0])
def test_c2_flat_1m_768_nq1024(gpu, c2_data, c2_oracle, form):
    """C2: 1M × 768, nq = 1024, k = 10 through hipann_flat_search_device (the bench's call), every
    fp32-level form; the oracle's BLAS-path top-k on all 1024 queries (the exact forms' direct-form distances
    order a near-tie differently from the BLAS form only inside the tie window); all rows sorted and distinct."""
    import torch

    xb_t, xq_t, xb, xq = c2_data
    ix = gpu.HipIndexFlatDevice(768, 0, xb_t.data_ptr(), xb_t.shape[0], 0, copy=False)
    ix.form = form
    D, I = _dev_search(ix, xq_t, 10, torch)
    Do, Io = c2_oracle
    st = check_topk_parity(xb, xq, D, I, Do, Io, 0)
    assert st["exact_fraction"] >= (0.999 if form in (3, 4, 5) else 0.995), st
    assert np.all(np.diff(D, axis=1) >= 0) and np.all(I >= 0)
    assert all(len(set(r)) == 10 for r in I.tolist())
    ix.close()


def test_c2_flat_1m_768_request_k30(gpu, c2_data, oracle):
    """C2 with request_k = 30 (k = 10 plus 20 tombstones, faiss_index.cpp:713-715): the bounded passes with a
    64-candidate int8 filter (the default form), exact; the oracle's parity rule on 256 queries."""
    import torch

    xb_t, xq_t, xb, xq = c2_data
    ix = gpu.HipIndexFlatDevice(768, 0, xb_t.data_ptr(), xb_t.shape[0], 0, copy=False)
    D, I = _dev_search(ix, xq_t, 30, torch)
    assert ix.last_search_path() == {"form": 5, "filter_k": 64, "sublists": 0}
    Do, Io = oracle.flat_search(xb, xq[:256], 30, 0)
    st = check_topk_parity(xb, xq[:256], D[:256], I[:256], Do, Io, 0)
    assert st["exact_fraction"] >= 0.995, st
    assert ix.rerank_fallbacks() == 0
    ix.close()


@pytest.fixture(scope="module")
def c3_index(gpu):
    import torch

    import bench
    from ivf_build import build_ivf_shard

    dev = torch.device("cuda", 0)
    n, d, nq, nlist, nprobe = 200_000, 768, 1024, 1024, 32
    gc = torch.Generator(device=dev).manual_seed(7)
    basis = bench.lowrank_basis(torch, 16, d, gc)  # the bench's C3 data model (intrinsic dim 16)
    xb_t = torch.empty((n, d), device=dev, dtype=torch.float32)
    bench.gen_lowrank_rows(torch, xb_t, 0, basis, 0.02, 42)
    xq_t = torch.empty((nq, d), device=dev, dtype=torch.float32)
    bench.gen_lowrank_rows(torch, xq_t, 0, basis, 0.02, 4242)
    xb = xb_t.cpu().numpy()
    index, info = build_ivf_shard(torch, gpu, xb_t, 0, n, nlist, nprobe, 0, 0, 1, centres_seed=1234)
    del xb_t
    cen_t, codes_t, ids_t = index._keep
    lists = (cen_t.cpu().numpy(), index._offsets.copy(), ids_t.cpu().numpy(), codes_t.cpu().numpy())
    return index, info, xb, xq_t, xq_t.cpu().numpy(), lists


@pytest.fixture(scope="module")
def c3_oracle(c3_index, oracle):
    _, _, _, _, xq, (cen, off, ids, codes) = c3_index
    return oracle.ivf_search(cen, off, ids, codes, xq, 10, 32, 0)


@pytest.mark.parametrize("form", [6, 5, 3, 0])
def test_c3_ivf_nlist1024_nprobe32_d768_nq1024(gpu, oracle, c3_index, c3_oracle, form):
    """C3 shape: nlist = 1024, nprobe = 32, d = 768, nq = 1024, k = 10 (200k rows of the bench's data,
    lists from the bench's GPU build).  Probe lists equal the oracle's; ids follow the parity rule over
    the scanned set on every query whose probe list is identical (tie-window differences excluded)."""
    import torch

    index, info, xb, xq_t, xq, (cen, off, ids, codes) = c3_index
    assert info["nlist"] == 1024 and np.diff(off).sum() == len(xb)
    index.form = form
    D, I = _dev_search(index, xq_t, 10, torch)
    P = index.last_probes(len(xq))
    Do, Io, Po = c3_oracle
    # every query checked: a probe list that differs from the oracle's (inside the coarse tie window only) is held to
    # the oracle's search_preassigned over the GPU's list; SURVEY §8c: identical probe lists — the count must be 0
    Do, Io, ndiff = oracle_on_gpu_probes(oracle, cen, off, ids, codes, xq, 10, P, Po, Do, Io, 0)
    assert ndiff <= C3_MAX_PROBE_DIFF, ndiff
    st = check_topk_parity(xb, xq, D, I, Do, Io, 0)
    assert st["exact_fraction"] >= (1.0 if form in (5, 6) else 0.995), st
    if form in (5, 6):  # returned distances are the direct fp32 form, like the oracle's scanner
        v = I >= 0
        assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)
    index.form = 6


def test_c3_ivf_2m_rows_full_batch_vs_oracle(gpu, oracle):
    """C3 at 2M rows (nlist 1024, nprobe 32, d 768, the bench's data model and GPU build), the whole 1024-query
    batch against the oracle's IndexIVFFlat::search: probe lists identical, ids and order identical on every query
    with an identical probe list (exact_fraction 1.0), returned distances equal the oracle's direct-form fp32 ones."""
    import torch

    import bench
    from ivf_build import build_ivf_shard

    dev = torch.device("cuda", 0)
    n, d, nq, nlist, nprobe = 2_000_000, 768, 1024, 1024, 32
    gc = torch.Generator(device=dev).manual_seed(7)
    basis = bench.lowrank_basis(torch, 16, d, gc)
    xb_t = torch.empty((n, d), device=dev, dtype=torch.float32)
    bench.gen_lowrank_rows(torch, xb_t, 0, basis, 0.02, 42)
    xq_t = torch.empty((nq, d), device=dev, dtype=torch.float32)
    bench.gen_lowrank_rows(torch, xq_t, 0, basis, 0.02, 4242)
    xb = xb_t.cpu().numpy()
    index, info = build_ivf_shard(torch, gpu, xb_t, 0, n, nlist, nprobe, 0, 0, 1, centres_seed=1234)
    del xb_t
    cen_t, codes_t, ids_t = index._keep
    cen, off, ids, codes = cen_t.cpu().numpy(), index._offsets.copy(), ids_t.cpu().numpy(), codes_t.cpu().numpy()
    xq = xq_t.cpu().numpy()
    D, I = _dev_search(index, xq_t, 10, torch)
    assert index.last_search_path()["form"] == index.FORM_HALF_EXACT
    P = index.last_probes(nq)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, nprobe, 0)
    Do, Io, ndiff = oracle_on_gpu_probes(oracle, cen, off, ids, codes, xq, 10, P, Po, Do, Io, 0)
    assert ndiff <= C3_MAX_PROBE_DIFF, ndiff
    st = check_topk_parity(xb, xq, D, I, Do, Io, 0)
    assert st["exact_fraction"] == 1.0, st
    v = I >= 0
    assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)
    index.close()


def test_c3_ivf_train_c_abi_recall(gpu, c3_index):
    """SURVEY §8f rank 4 at the C3 shape: the index built on centroids from the C ABI's training
    (hipann_ivf_train_device, used by ivf_build / the bench) reaches a recall@10 at nprobe 32 no worse than the
    same build with the r01-r03 torch k-means (ivf_build.kmeans_torch), against exact Flat on the same rows."""
    import torch

    import bench
    from ivf_build import build_ivf_shard, flat_ground_truth, kmeans_torch

    index, info, xb, xq_t, xq, _ = c3_index  # built through the C ABI's training
    gt = flat_ground_truth(torch, gpu, 768, 0, xq_t, 10, len(xb), 0, 1, ivf_info_tensor=index)
    _, I = _dev_search(index, xq_t, 10, torch)
    r_hip = bench.recall_at(I, gt, 10)
    xb_t = torch.from_numpy(xb).cuda()
    index_t, _ = build_ivf_shard(torch, gpu, xb_t, 0, len(xb), 1024, 32, 0, 0, 1, centres_seed=1234,
                                 train=kmeans_torch)
    del xb_t
    _, It = _dev_search(index_t, xq_t, 10, torch)
    r_torch = bench.recall_at(It, gt, 10)
    index_t.close()
    assert r_hip >= r_torch - 0.005, (r_hip, r_torch)
    assert r_hip >= 0.85, r_hip  # 200k rows over 1024 lists (≈195 per list) at nprobe 32


@pytest.mark.parametrize("form", [6, 5])
def test_c3_request_k30(gpu, c3_index, oracle, form):
    """C3 shape with request_k = 30 (k = 10 plus 20 tombstones): sub-list slots and a 60-candidate rerank,
    exact fp32 direct-form distances; ids follow the oracle's parity rule on every query whose probe list is
    the oracle's."""
    import torch

    index, info, xb, xq_t, xq, (cen, off, ids, codes) = c3_index
    index.form = form
    D, I = _dev_search(index, xq_t, 30, torch)
    assert index.last_search_path() == {"form": form, "filter_k": 60, "sublists": 8}
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 30, 32, 0)
    same = check_probe_parity(cen, xq, index.last_probes(len(xq)), Po, 0)
    st = check_topk_parity(xb, xq[same], D[same], I[same], Do[same], Io[same], 0)
    assert st["exact_fraction"] >= 0.995, st
    v = I[same] >= 0
    assert np.allclose(D[same][v], Do[same][v], rtol=2e-6, atol=1e-6)
    index.form = 6


@pytest.mark.parametrize("form", [6, 5])
def test_c3_duplicate_rows_faiss_tie_order(gpu, c3_index, oracle, form):
    """C3 shape with exact ties: every stored row of the C3 lists appears twice more in its list (the copies
    in reversed row order) under scattered labels — 600k rows, nlist 1024, nprobe 32, d 768, nq 1024.  FAISS's
    IVF scanner keeps, among rows tied at the 10th distance, the smallest labels among the earliest tied rows
    in scan order; the GPU (rerank, or the device fallback for flagged queries) must equal the oracle slot for
    slot on every query whose probe list is the oracle's (reference edge case: duplicates,
    test/sql/edge_cases.test:75-83)."""
    import torch

    index0, info, xb, xq_t, xq, (cen, off0, ids0, codes0) = c3_index
    nlist = len(cen)
    off = off0 * 3
    parts = []
    for l in range(nlist):
        c = codes0[off0[l]:off0[l + 1]]
        parts += [c, c[::-1], c]
    codes = np.ascontiguousarray(np.concatenate(parts))
    rng = np.random.default_rng(11)
    labels = (rng.permutation(len(codes)).astype(np.int64) * 5 + 3)
    ix = gpu.HipIndexIVFFlat(cen, off, labels, codes, 32, 0)
    ix.form = form
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, labels, codes, xq, 10, 32, 0)
    same = check_probe_parity(cen, xq, ix.last_probes(len(xq)), Po, 0)
    assert same.mean() >= 0.99, same.mean()
    exact = float((I[same] == Io[same]).mean())
    assert exact == 1.0, f"{(I[same] != Io[same]).any(axis=1).sum()} queries differ"
    v = I[same] >= 0
    assert np.allclose(D[same][v], Do[same][v], rtol=2e-6, atol=1e-6)
    ix.close()


def _c4_graph(gpu, n, d, R, seed, integer=False):
    import torch

    import bench
    import diskann_build as DB

    dev = torch.device("cuda", 0)
    gc = torch.Generator(device=dev).manual_seed(seed)
    if integer:
        g = torch.Generator(device=dev).manual_seed(seed)
        base = torch.randint(0, 4, (n // 4, d), generator=g, device=dev).to(torch.float32)
        x = base.repeat_interleave(4, 0)[torch.randperm(n, generator=g, device=dev)].contiguous()
        x[0] = 0.0
        x[1] = 255.0  # SQ8 min 0, scale 255: codes equal the values, distances exact in fp32
        q = torch.randint(0, 4, (256, d), generator=g, device=dev).to(torch.float32)
    else:
        basis = bench.lowrank_basis(torch, 16, d, gc)  # the bench's C4 data model
        x = torch.empty((n, d), device=dev, dtype=torch.float32)
        bench.gen_lowrank_rows(torch, x, 0, basis, 0.02, 42)
        q = torch.empty((512, d), device=dev, dtype=torch.float32)
        bench.gen_lowrank_rows(torch, q, 0, basis, 0.02, 4242)
    codes, mins, scale = DB.sq8_encode(torch, x)
    adj_t, medoid = DB.knn_graph(torch, x, R=R, n_random=R // 4, seed=seed)
    adj = DB.adjacency_u32(torch, adj_t)
    torch.cuda.synchronize()
    return (x.cpu().numpy(), q.cpu().numpy(), codes.cpu().numpy(), mins.cpu().numpy(), scale.cpu().numpy(), adj,
            medoid)


@pytest.mark.parametrize("metric", [0, 1])
def test_c4_resident_bfs_d1536_sq8_L128(gpu, oracle, metric):
    """C4 shape: the resident traversal at d = 1536 SQ8, R = 64, L = 128 (the bench's template of
    diskann_bfs) on a 32k-node graph from the bench's builder, vs DiskProvider::search_batch restated.
    The device SQ8 encoder equals the oracle's codec; BFS ids ≥ 99% identical (summation order can
    move a trajectory), distances within 1e-5, evaluation counts within 1%."""
    x, q, codes, mins, scale, adj, medoid = _c4_graph(gpu, 32768, 1536, 64, 8)
    m2, s2 = oracle.sq8_train(x)
    assert np.array_equal(mins, m2) and np.array_equal(scale, s2)
    assert np.array_equal(codes, oracle.sq8_encode(x, mins, scale))
    db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
    db.register_graph(adj)
    ids, dists, st = db.search_batch_resident([medoid], q, 10, 128, metric)
    assert st["host_requeries"] == 0 and st["pops"] > 0
    oi, od, ost = oracle.diskann_search_batch(adj, [medoid], q, 10, 128, metric, codes=codes, mins=mins,
                                               scale=scale)
    assert (ids == oi).mean() >= 0.99
    same = ids == oi
    assert np.allclose(dists[same], od[same], rtol=1e-5, atol=1e-4)
    assert abs(st["evals"] - ost["evals"]) <= 0.01 * ost["evals"]
    assert np.all(np.diff(dists, axis=1) >= 0)
    # the host lock-step BFS over the id-gather kernel (the reference-shaped path) on the same graph
    hi, hd, hst = db.search_batch(adj, [medoid], q[:128], 10, 128, metric)
    assert (hi == oi[:128]).mean() >= 0.99


def test_c4_resident_bfs_d1536_exact_ties(gpu, oracle):
    """C4 shape on small-integer data (every distance exact in fp32, rows duplicated 4×: exact ties in the
    result-list binary search, the boundary evictions and the spill list): ids, distances, evaluation
    and step counts identical to the oracle."""
    x, q, codes, mins, scale, adj, medoid = _c4_graph(gpu, 16384, 1536, 64, 9, integer=True)
    assert np.all(mins == 0) and np.all(scale == 255)
    db = gpu.DiskannDeviceDB(codes, 1, mins, scale)
    db.register_graph(adj)
    ids, dists, st = db.search_batch_resident([medoid, 7], q, 10, 128)
    oi, od, ost = oracle.diskann_search_batch(adj, [medoid, 7], q, 10, 128, 0, codes=codes, mins=mins, scale=scale)
    assert np.array_equal(ids, oi)
    assert np.array_equal(dists, od)
    assert st["evals"] == ost["evals"]
    assert st["steps"] == ost["steps"]
