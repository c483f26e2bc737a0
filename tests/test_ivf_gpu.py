"""GPU parity tests of the IVFFlat path against the oracle (FAISS IndexIVFFlat::search restatement).

Given identical centroids and inverted lists, the GPU must choose identical probe lists and return the
oracle's ids under the Flat parity rule over the scanned set.  Shapes follow
faiss-metal/tests/test_metal_ivfflat.mm:28-166 (nv=2000, d=64, nlist=16, nprobe=4).
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

from _data import SPLIT2_TAU, TAU, build_ivf_lists, check_topk_parity, faiss_metal_case

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
SQL = json.loads((GOLD / "sql_known_answers.json").read_text())
sys.path.insert(0, str(GOLD))
from make_golden import IVF_CASES  # noqa: E402


def _tol(form):
    """Parity windows: fp32-level forms use the calibrated tau; form 4 (2-term split, measurement only)
    its proven error bound (tests/_data.py SPLIT2_TAU)."""
    return dict(tau=SPLIT2_TAU, dist_tau=SPLIT2_TAU) if form == 4 else dict(tau=TAU)


def _ivf(gpu, xb, nlist, nprobe, metric=0, devices=None, stride=None):
    cen = np.ascontiguousarray(xb[:: (stride or len(xb) // nlist)][:nlist])
    off, ids, codes = build_ivf_lists(xb, cen, metric)
    return gpu.HipIndexIVFFlat(cen, off, ids, codes, nprobe, metric, devices=devices), (cen, off, ids, codes)


@pytest.mark.parametrize("nv,d,nlist,nprobe,nq,k,metric", IVF_CASES)
def test_ivf_faiss_metal_shapes(gpu, oracle, nv, d, nlist, nprobe, nq, k, metric):
    xb, xq = faiss_metal_case(nv, nq, d)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, nlist, nprobe, metric)
    D, I = ix.search(xq, k)
    z = np.load(GOLD / "ivf_mt19937.npz")
    key = f"ivf_{nv}_{d}_{nlist}_{nprobe}_{nq}_{k}_{metric}"
    assert np.array_equal(ix.last_probes(nq), z[key + "_P"].astype(np.int64))
    check_topk_parity(xb, xq, D, I, z[key + "_D"], z[key + "_I"].astype(np.int64), metric)


@pytest.mark.parametrize("nq", [1, 7, 19, 20, 64, 333])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4, 5, 6, 7])
def test_ivf_vs_oracle_probe_sets(gpu, oracle, nq, metric, form):
    xb, xq = faiss_metal_case(20000, nq, 96)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 64, 8, metric)
    ix.form = form
    assert ix.form == form
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 8, metric)
    assert np.array_equal(ix.last_probes(nq), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric, **_tol(form))


@pytest.mark.parametrize("d", [4, 8, 12, 20, 44, 77, 132, 768])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4, 5, 6, 7])
def test_ivf_dims(gpu, oracle, d, metric, form):
    """Dimensions around the scans' LDS chunks (32 dims MFMA, 32 VALU-decomposed, 24 direct: partial
    last chunk, d < one chunk) and d % 4 != 0 (the decomposed forms fall back to the direct kernel)."""
    xb, xq = faiss_metal_case(3000, 40, d)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 8, 3, metric)
    ix.form = form
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 3, metric)
    assert np.array_equal(ix.last_probes(40), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric, **_tol(form))


@pytest.mark.parametrize("nq", [5, 70])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4, 5, 6, 7])
def test_ivf_long_lists(gpu, oracle, nq, form):
    """Lists longer than one work item's row chunk (2048 rows) and ragged 256-row tiles; with nq = 70 a
    list's probing queries split over several query groups."""
    xb, xq = faiss_metal_case(21000, nq, 64)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 4, 2)
    ix.form = form
    assert np.diff(off).max() > 2048
    D, I = ix.search(xq, 20)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 20, 2, 0)
    assert np.array_equal(ix.last_probes(nq), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, **_tol(form))


@pytest.mark.parametrize("nq", [1, 15, 16, 17, 31, 33, 47, 48, 49, 64, 65, 130])
@pytest.mark.parametrize("d,metric", [(96, 0), (100, 0), (96, 1)])
@pytest.mark.parametrize("form", [0, 3, 4, 5, 6, 7])
def test_ivf_mfma_query_tiles(gpu, oracle, nq, d, metric, form):
    """One list probed by every query: items of 1-4 16-query tiles (every wave → work mapping of the
    MFMA scan, incl. the idle wave at 3 tiles and the list merges at 1-2 tiles), several query groups
    (nq > 64), 3 row chunks with a ragged last tile, and a partial last 32-dim chunk (d = 100)."""
    xb, xq = faiss_metal_case(5000, nq, d)
    cen = np.ascontiguousarray(xb[:1])
    off = np.array([0, len(xb)], np.int64)
    ids = np.arange(len(xb), dtype=np.int64)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, xb, 1, metric)
    ix.form = form
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, xb, xq, 10, 1, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric, **_tol(form))


@pytest.mark.parametrize("nq", [17, 49, 80, 81, 96, 97, 150, 193, 256, 257, 290, 513, 700])
@pytest.mark.parametrize("d,metric", [(96, 0), (100, 1), (768, 0), (1536, 0)])
@pytest.mark.parametrize("k", [10, 20])
@pytest.mark.parametrize("form", [6, 7])
def test_ivf_half_wide_items(gpu, oracle, nq, d, metric, k, form):
    """The fp16 form's one-term items (ivf_mfma.hip): every list's queries enter on their high fp16 term, in wide
    items of up to 96 queries (48 at d = 1536): one item of 17-96 queries (2-6 query tiles), two of 48/49 or 128/129,
    three or more, ragged last query tiles; k = 20 takes the sub-list slots.  Run with HIPANN_IVF_GEMM=1 (A/B,
    tools/gpu_r06_gemm.sh) a list probed by more than 96 queries takes GEMM items of up to 256 instead (one of 97-256
    queries, two of 128/129, three of 171 at 513).  The rerank bounds those queries with their one-term residual, so
    the ids still equal the oracle's.  Form 7 (the int8 image) runs the same items over 64-dim super-steps (96 queries
    at d = 1536 too) with the sub-lists and 64 reranked candidates at every k."""
    xb, xq = faiss_metal_case(4500 if d < 1000 else 2500, nq, d)
    cen = np.ascontiguousarray(xb[:2])
    off = np.array([0, 2100, len(xb)], np.int64)  # two lists, both probed by every query: 2 row chunks, ragged
    ids = np.arange(len(xb), dtype=np.int64)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, xb, 2, metric)
    ix.form = form
    D, I = ix.search(xq, k)
    assert ix.last_search_path()["form"] == form
    Do, Io, Po = oracle.ivf_search(cen, off, ids, xb, xq, k, 2, metric)
    assert np.array_equal(ix.last_probes(nq), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric, tau=TAU)


def test_ivf_full_probe_equals_flat(gpu, oracle):
    xb, xq = faiss_metal_case(6000, 50, 48)
    ix, _ = _ivf(gpu, xb, 32, 32)
    D, I = ix.search(xq, 10)
    fl = gpu.HipIndexFlat(48, 0, xb)
    Df, If = fl.search(xq[:10], 10)       # direct form, like the IVF scan (summation order differs)
    assert (I[:10] == If).mean() > 0.99
    assert np.allclose(D[:10], Df, rtol=1e-5, atol=1e-5)
    Do, Io = oracle.flat_search(xb, xq, 10)
    check_topk_parity(xb, xq, D, I, Do, Io)


def test_ivf_sql_known_answer(gpu):
    case = SQL["faiss_ivfflat_exact"]
    xb = np.array(case["xb"], np.float32)
    cen = xb[[0, 4]].copy()
    off, ids, codes = build_ivf_lists(xb, cen)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, codes, case["nprobe"])
    for qc in case["queries"]:
        D, I = ix.search(np.array([qc["q"]], np.float32), qc["k"])
        assert I[0].tolist() == qc["ids"]
        if "dists" in qc:
            assert np.allclose(D[0], qc["dists"])


def test_ivf_edge_cases(gpu, oracle):
    xb, xq = faiss_metal_case(3000, 25, 40)
    cen = np.ascontiguousarray(xb[:20])
    off, ids, codes = build_ivf_lists(xb, cen)
    # add empty lists: centroids far away
    cen2 = np.vstack([cen, np.full((4, 40), 50.0, np.float32)])
    off2 = np.concatenate([off, np.full(4, off[-1])])
    ix = gpu.HipIndexIVFFlat(cen2, off2, ids, codes, 30)  # nprobe > nlist → clamped (IndexIVF::search)
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen2, off2, ids, codes, xq, 10, 30)
    assert np.array_equal(ix.last_probes(25), Po)
    check_topk_parity(xb, xq, D, I, Do, Io)
    # k larger than the scanned set → pads
    ix.nprobe = 1
    D, I = ix.search(xq[:3], 64)
    Do, Io, _ = oracle.ivf_search(cen2, off2, ids, codes, xq[:3], 64, 1)
    assert np.array_equal(I < 0, Io < 0)
    # empty index
    e = gpu.HipIndexIVFFlat(cen, np.zeros(21, np.int64), np.zeros(0, np.int64), np.zeros((0, 40), np.float32), 4)
    D, I = e.search(xq[:2], 5)
    assert (I == -1).all()
    with pytest.raises(gpu.HipAnnError):
        ix.search(xq[:1], 0)
    with pytest.raises(gpu.HipAnnError):
        ix.nprobe = 0


def test_ivf_labels_are_stored_ids(gpu, oracle):
    """index_cpu_to_metal_ivf copies per-list ids; results are those labels (MetalIndexIVFFlat.mm:243-250)."""
    xb, xq = faiss_metal_case(2000, 8, 32)
    cen = np.ascontiguousarray(xb[::200][:10])
    off, ids, codes = build_ivf_lists(xb, cen)
    labels = ids * 7 + 1_000_000_000_000  # arbitrary int64 labels
    ix = gpu.HipIndexIVFFlat(cen, off, labels, codes, 10)
    D, I = ix.search(xq, 5)
    Do, Io, _ = oracle.ivf_search(cen, off, labels, codes, xq, 5, 10)
    assert np.array_equal(I, Io)


def test_ivf_multi_shard_same_device(gpu, oracle):
    xb, xq = faiss_metal_case(8000, 40, 64)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 32, 6, devices=[0, 0])
    D, I = ix.search(xq, 10)
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 6)
    check_topk_parity(xb, xq, D, I, Do, Io)


def test_ivf_backend_and_device_api(gpu, oracle):
    import torch
    xb, xq = faiss_metal_case(10000, 100, 128)
    cen = np.ascontiguousarray(xb[::100][:100])
    off, ids, codes = build_ivf_lists(xb, cen)
    g = gpu.get_gpu_backend().cpu_to_gpu({"type": "IVFFlat", "centroids": cen, "list_offsets": off, "ids": ids,
                                          "codes": codes, "nprobe": 8})
    D, I = g.search(xq, 10)
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 8)
    check_topk_parity(xb, xq, D, I, Do, Io)
    dev = torch.device("cuda", 0)
    c_t, i_t, x_t = (torch.from_numpy(a).to(dev) for a in (cen, ids, codes))
    q_t = torch.from_numpy(xq).to(dev)
    ix = gpu.HipIndexIVFFlat.from_device(128, 0, 100, 8, c_t.data_ptr(), off, i_t.data_ptr(), x_t.data_ptr(), 0)
    Dt = torch.empty((100, 10), device=dev)
    It = torch.empty((100, 10), device=dev, dtype=torch.int64)
    ix.search_device(100, q_t.data_ptr(), 10, Dt.data_ptr(), It.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(It.cpu().numpy(), I) and np.array_equal(Dt.cpu().numpy(), D)


@pytest.mark.parametrize("eager", [False, True])
def test_ivf_device_api_alternating_streams(gpu, eager):
    """Consecutive calls on one handle from different streams (StreamFence): a call on a new stream may not start
    before the previous call's kernels are done with the shard's scratch (lazy default: a device synchronisation on
    a stream switch; HIPANN_FENCE_EAGER=1: per-call events, run in a child process).  Each batch's answers equal the
    same batch searched alone."""
    import subprocess
    import torch
    if eager:
        code = ("import sys; sys.path.insert(0, %r); import test_ivf_gpu as t; t._alternating_streams_body()"
                % str(Path(__file__).resolve().parent))
        env = dict(os.environ, HIPANN_FENCE_EAGER="1")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return
    _alternating_streams_body()


def _alternating_streams_body():
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "duckdb-annsearch_amd"))
    import hipann as gpu
    rng = np.random.default_rng(11)
    d, n, nlist = 64, 40000, 64
    xb = rng.standard_normal((n, d)).astype(np.float32)
    cen = np.ascontiguousarray(xb[:: n // nlist][:nlist])
    off, ids, codes = build_ivf_lists(xb, cen)
    dev = torch.device("cuda", 0)
    c_t, i_t, x_t = (torch.from_numpy(a).to(dev) for a in (cen, ids, codes))
    ix = gpu.HipIndexIVFFlat.from_device(d, 0, nlist, 8, c_t.data_ptr(), off, i_t.data_ptr(), x_t.data_ptr(), 0)
    batches = [torch.from_numpy(rng.standard_normal((512, d)).astype(np.float32)).to(dev) for _ in range(6)]
    ref = []
    for q in batches:  # each batch alone, synchronised
        D = torch.empty((512, 10), device=dev)
        I = torch.empty((512, 10), device=dev, dtype=torch.int64)
        ix.search_device(512, q.data_ptr(), 10, D.data_ptr(), I.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    outs = []
    for j, q in enumerate(batches):  # back to back, alternating streams, no host synchronisation in between
        s = streams[j % 2]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            D = torch.empty((512, 10), device=dev)
            I = torch.empty((512, 10), device=dev, dtype=torch.int64)
            ix.search_device(512, q.data_ptr(), 10, D.data_ptr(), I.data_ptr(), s.cuda_stream)
        outs.append((D, I))
    torch.cuda.synchronize()
    for (D, I), (Dr, Ir) in zip(outs, ref):
        assert np.array_equal(I.cpu().numpy(), Ir) and np.array_equal(D.cpu().numpy(), Dr)


def test_ivf_gpu_build_recall(gpu):
    """ivf_build (GPU k-means + assignment + list sort) on clustered data: recall@10 vs exact ≥ 0.95."""
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from ivf_build import build_ivf_shard, flat_ground_truth
    import bench
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    d, n = 64, 200_000
    centres = torch.rand((256, d), generator=g, device=dev) * 2 - 1
    xb = torch.empty((n, d), device=dev)
    bench.gen_clustered_rows(torch, xb, 0, centres, 0.25, 42)
    a = torch.randint(0, 256, (200,), generator=g, device=dev)
    xq = (centres[a] + torch.randn((200, d), generator=g, device=dev) * 0.25).contiguous()
    ix, info = build_ivf_shard(torch, gpu, xb, 0, n, 64, 8, 0, 0, 1)
    stream = torch.cuda.current_stream().cuda_stream
    D = torch.empty((200, 10), device=dev)
    I = torch.empty((200, 10), device=dev, dtype=torch.int64)
    ix.search_device(200, xq.data_ptr(), 10, D.data_ptr(), I.data_ptr(), stream)
    gt = flat_ground_truth(torch, gpu, d, 0, xq, 10, n, 0, 1, ivf_info_tensor=ix)
    got = I.cpu().numpy()
    recall = np.mean([len(set(got[i]) & set(gt[i])) / 10 for i in range(200)])
    assert recall >= 0.95, recall
    assert info["list_size_min"] >= 0 and sum(np.diff(ix._offsets)) == n


@pytest.mark.parametrize("k", [65, 100, 257, 1000])
@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_large_k(gpu, oracle, k, metric):
    """k > 64 (faiss-metal selects up to k = 2048, MetalSelect.mm:31-74): the per-slot scan + LDS sort
    path, lists longer than one 2048-row chunk (a probed list contributes several slots), k larger
    than some probed lists and than a chunk tail."""
    xb, xq = faiss_metal_case(12000, 37, 40)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 8, 3, metric)
    D, I = ix.search(xq, k)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, k, 3, metric)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)


@pytest.mark.parametrize("nprobe", [65, 100, 256])
@pytest.mark.parametrize("k", [10, 64])
def test_ivf_large_nprobe(gpu, oracle, nprobe, k):
    """nprobe > 64 (the coarse quantizer takes the Flat large-k path); nprobe = nlist equals Flat."""
    xb, xq = faiss_metal_case(30000, 50, 32)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 256, nprobe)
    D, I = ix.search(xq, k)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, k, nprobe)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(xb, xq, D, I, Do, Io)
    if nprobe == 256:
        Df, If_ = oracle.flat_search(xb, xq, k)
        check_topk_parity(xb, xq, D, I, Df, If_)


@pytest.mark.parametrize("form", [5, 6, 7])
@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_exact_form_distances_are_direct(gpu, oracle, metric, form):
    """Forms 5 and 6 (default): the returned distances are the direct-form fp32 distances of the returned
    rows (FAISS CPU IVFFlatScanner arithmetic; only the summation order differs), and the ids follow the
    oracle's (distance, label) order."""
    xb, xq = faiss_metal_case(20000, 64, 96)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 64, 8, metric)
    assert ix.form == 6  # the library default
    ix.form = form
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 8, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    valid = I >= 0
    assert np.allclose(D[valid], Do[valid], rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("form", [5, 6, 7])
def test_ivf_exact_form_fallback_on_ties(gpu, oracle, form):
    """Every vector stored 24 times: the 16 rerank candidates tie, the bound check cannot prove the top-k,
    and the flagged queries are re-run on the device in the direct form — results equal the oracle's, slot for
    slot (FAISS's scan-order admission of exact ties)."""
    base, xq = faiss_metal_case(600, 40, 64)
    xb = np.ascontiguousarray(np.repeat(base, 24, axis=0))
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 16, 4, 0)
    ix.form = form
    before = ix.rerank_fallbacks()
    D, I = ix.search(xq, 10)
    assert ix.rerank_fallbacks() > before
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 4, 0)
    assert np.array_equal(ix.last_probes(40), Po)
    st = check_topk_parity(xb, xq, D, I, Do, Io, 0)
    assert st["exact_fraction"] == 1.0, st


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_ivf_add_on_gpu_copy(gpu, oracle, devices):
    """IndexIVFFlat::add_with_ids on the GPU copy (hipann_ivf_add): appended rows land in their nearest
    centroid's list after the existing rows (insertion order), labels given or ntotal + i; the exported
    lists equal the oracle's assignment of all rows, and search keeps parity."""
    xb, xq = faiss_metal_case(9000, 30, 48)
    cen = np.ascontiguousarray(xb[::300][:30])
    n1 = 5000
    off1, ids1, codes1 = build_ivf_lists(xb[:n1], cen)
    ix = gpu.HipIndexIVFFlat(cen, off1, ids1, codes1, 6, devices=devices)
    ix.search(xq, 10)  # builds the scan's tiled copy, which the add must invalidate
    ix.add(xb[n1:8000])                      # labels ntotal + i
    ix.add(xb[8000:8010])                    # < 20 rows: FAISS assigns with the direct form
    ix.add(xb[8010:], ids=np.arange(8010, 9000, dtype=np.int64))
    assert ix.ntotal == 9000
    ex = ix.export()
    off, ids, codes = build_ivf_lists(xb, cen)
    assert np.array_equal(ex["list_offsets"], off)
    assert np.array_equal(ex["ids"], ids) and np.array_equal(ex["codes"], codes)
    assert np.array_equal(ex["centroids"], cen)
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 6)
    assert np.array_equal(ix.last_probes(30), Po)
    check_topk_parity(xb, xq, D, I, Do, Io)


def test_ivf_search_per_call_nprobe_threads(gpu, oracle):
    """hipann_ivf_search_np: concurrent searches with different nprobe on one handle (two DuckDB
    connections with different SearchParametersIVF) each get their own nprobe; the index's own nprobe
    is unchanged."""
    import threading
    xb, xq = faiss_metal_case(8000, 40, 32)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 40, 2)
    ref = {np_: oracle.ivf_search(cen, off, ids, codes, xq, 10, np_)[1] for np_ in (1, 3, 9, 40)}
    errors = []

    def run(np_):
        for _ in range(5):
            _, I = ix.search(xq, 10, nprobe=np_)
            if not np.array_equal(I, ref[np_]):
                errors.append(np_)

    ts = [threading.Thread(target=run, args=(p,)) for p in (1, 3, 9, 40) for _ in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors
    assert ix.nprobe == 2 and gpu.lib().hipann_ivf_get_nprobe(ix._h) == 2


def test_ivf_gpu_to_cpu_round_trip(gpu, oracle):
    """GpuBackend::GpuToCpu for IVFFlat (gpu_backend_metal.mm:62-67): the exported CPU index equals the
    one converted in, and converting it back searches identically."""
    be = gpu.get_gpu_backend()
    xb, xq = faiss_metal_case(6000, 25, 40)
    cen = np.ascontiguousarray(xb[::200][:30])
    off, ids, codes = build_ivf_lists(xb, cen)
    cpu = {"type": "IVFFlat", "centroids": cen, "list_offsets": off, "ids": ids * 3 + 11, "codes": codes,
           "nprobe": 5, "metric": 0}
    g = be.cpu_to_gpu(cpu)
    back = be.gpu_to_cpu(g)
    for key in ("centroids", "list_offsets", "ids", "codes"):
        assert np.array_equal(back[key], cpu[key]), key
    assert back["nprobe"] == 5 and back["metric"] == 0 and back["type"] == "IVFFlat"
    g2 = be.cpu_to_gpu(back)
    assert all(np.array_equal(a, b) for a, b in zip(g.search(xq, 10), g2.search(xq, 10)))


def test_ivf_label_int32_max_survives_multi_shard_merge(gpu, oracle):
    """Labels around 2^31 − 1 through the multi-shard int64 merge (merge_parts_topk<long long>): the int32
    partials' pad value must not drop a real int64 label 2147483647."""
    xb, xq = faiss_metal_case(3000, 12, 32)
    cen = np.ascontiguousarray(xb[::300][:10])
    off, ids, codes = build_ivf_lists(xb, cen)
    labels = ids + (2**31 - 1) - ids[np.argmin(np.abs(ids - 100))]  # some row carries exactly 2^31 - 1
    ix = gpu.HipIndexIVFFlat(cen, off, labels, codes, 10, devices=[0, 0])
    q = np.vstack([codes[np.nonzero(labels == 2**31 - 1)[0]], xq])
    D, I = ix.search(q, 5)
    Do, Io, _ = oracle.ivf_search(cen, off, labels, codes, q, 5, 10)
    assert I[0, 0] == 2**31 - 1
    assert np.array_equal(I, Io)


@pytest.mark.parametrize("scale,metric", [(1e6, 0), (1e-6, 0), (2.0 ** -112, 1), (2.0 ** 40, 1)])
def test_ivf_half_form_scaled_data(gpu, oracle, scale, metric):
    """Form 6 scales the rows by a power of two into fp16's range (x·2^(14-e)), so the fp16 image keeps
    its relative precision at any magnitude; codes whose scale leaves 2^±100 take form 5 instead.  Either
    way the results follow the oracle on the same (scaled) data."""
    xb, xq = faiss_metal_case(6000, 24, 64)
    xb = np.ascontiguousarray((xb.astype(np.float64) * scale).astype(np.float32))
    xq = np.ascontiguousarray((xq.astype(np.float64) * (scale if metric == 0 else 1.0)).astype(np.float32))
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 24, 6, metric)
    assert ix.form == 6
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 6, metric)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    v = I >= 0
    assert np.allclose(D[v], Do[v], rtol=2e-6, atol=0)


def test_ivf_half_form_query_out_of_range(gpu, oracle):
    """A query whose own scale leaves the fp16 form's safe range (here |q| ~ 2^110, IP) gets a non-finite
    bound: the rerank flags it and it is re-run on the device (direct form); the other queries are unaffected."""
    xb, xq = faiss_metal_case(6000, 24, 64)
    xq = xq.copy()
    xq[3] *= np.float32(2.0 ** 110)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 24, 6, 1)
    before = ix.rerank_fallbacks()
    D, I = ix.search(xq, 10)
    assert ix.rerank_fallbacks() - before >= 1
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 6, 1)
    check_topk_parity(xb, xq, D, I, Do, Io, 1)


@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_device_fallback_labels_and_batch(gpu, oracle, metric):
    """The device-side re-run of flagged queries (ivf_fallback_scan/_merge): every vector stored 20 times
    under scattered int64 labels, so most of a 300-query batch is flagged.  FAISS's IVF scanner keeps, of
    the rows tied at the k-th distance, the smallest labels among the EARLIEST tied rows in scan order (strict
    admission, (key, label) eviction) — not simply the smallest labels; the re-run reproduces that, so the
    result equals the oracle slot for slot (r02: 0.076 of the slots with (distance, label) order).  The flag
    count reaches rerank_fallbacks() without a host readback per batch.  Reference edge case: duplicates,
    test/sql/edge_cases.test:75-83."""
    base, xq = faiss_metal_case(500, 300, 48)
    xb = np.ascontiguousarray(np.repeat(base, 20, axis=0))
    cen = np.ascontiguousarray(xb[::500][:20])
    off, ids, codes = build_ivf_lists(xb, cen, metric)
    labels = np.ascontiguousarray((ids * 7919) % 100003 + 5, dtype=np.int64)
    ix = gpu.HipIndexIVFFlat(cen, off, labels, codes, 5, metric)
    before = ix.rerank_fallbacks()
    D, I = ix.search(xq, 10)
    assert ix.rerank_fallbacks() - before >= 100
    Do, Io, Po = oracle.ivf_search(cen, off, labels, codes, xq, 10, 5, metric)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    by_label = np.zeros((int(labels.max()) + 1, xb.shape[1]), np.float32)  # the parity rule indexes rows by label
    by_label[labels] = codes
    st = check_topk_parity(by_label, xq, D, I, Do, Io, metric)
    assert st["exact_fraction"] == 1.0, st
    v = I >= 0
    assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("form", [5, 6, 7])
@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_exact_ties_scan_order_unflagged(gpu, oracle, form, metric):
    """Exact ties that the rerank resolves itself (no fallback): each vector stored 3 times in its list, the
    copies in different row orders and under scattered labels, so the 10th distance is a 3-way tie while the
    16 candidates still prove the top-10 (the tie sits well inside the candidate list).  The rerank applies
    FAISS's scan-order rule (ivf_scan_order_topk) and the result equals the oracle slot for slot."""
    base, xq = faiss_metal_case(3000, 200, 64)
    cen = np.ascontiguousarray(base[::150][:20])
    off0, ids0, codes0 = build_ivf_lists(base, cen, metric)
    rng = np.random.default_rng(5)
    off = off0 * 3
    codes = np.concatenate([np.concatenate([codes0[off0[l]:off0[l + 1]], codes0[off0[l]:off0[l + 1]][::-1],
                                            codes0[off0[l]:off0[l + 1]]]) for l in range(len(cen))])
    labels = rng.permutation(len(codes)).astype(np.int64) * 3 + 11
    ix = gpu.HipIndexIVFFlat(cen, off, labels, np.ascontiguousarray(codes), 5, metric)
    ix.form = form
    before = ix.rerank_fallbacks()
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, labels, np.ascontiguousarray(codes), xq, 10, 5, metric)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    assert np.array_equal(I, Io), f"{(I != Io).any(axis=1).sum()} queries differ"
    v = I >= 0
    assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)
    # most queries were resolved by the rerank itself (the fallback covers the rest)
    assert ix.rerank_fallbacks() - before < len(xq) // 2


@pytest.mark.parametrize("form", [6, 5, 0, 7])
def test_ivf_successive_appends_incremental(gpu, oracle, form):
    """20 successive 2048-row appends (DuckDB's Append chunks, faiss_index.cpp:469) after the
    scan's tiled image exists.  Each append writes its rows into their lists' slack (ivf_relayout grows only the
    lists that overflow), re-tiles the touched passes and updates the bound maxima; the grown index exports the
    oracle's CSR lists and its ids equal the oracle's IndexIVFFlat::search on every query (exact forms: exactly)."""
    rng = np.random.default_rng(5 + form)
    d, nlist, n0, step, steps = 64, 64, 40_000, 2048, 20
    xb = rng.standard_normal((n0 + step * steps, d), dtype=np.float32)
    xb[-step:] *= np.float32(3.0)  # the last chunk raises max|x|, max‖x‖² and the residual maxima
    xq = rng.standard_normal((256, d), dtype=np.float32)
    xq[:16] = xb[-16:] + np.float32(1e-3)  # queries whose answers are the grown rows
    cen = np.ascontiguousarray(xb[:nlist * 50:50])
    off0, ids0, codes0 = build_ivf_lists(xb[:n0], cen)
    ix = gpu.HipIndexIVFFlat(cen, off0, ids0, codes0, 8)
    ix.form = form
    ix.search(xq, 10)  # builds the tiled image the appends must maintain
    for a in range(steps):
        lo = n0 + a * step
        ix.add(xb[lo:lo + step])
    assert ix.ntotal == len(xb)
    off, ids, codes = build_ivf_lists(xb, cen)
    ex = ix.export()
    assert np.array_equal(ex["list_offsets"], off) and np.array_equal(ex["ids"], ids)
    assert np.array_equal(ex["codes"], codes)
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == form
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 8)
    assert np.array_equal(ix.last_probes(256), Po)
    st = check_topk_parity(xb, xq, D, I, Do, Io)
    if form in (5, 6, 7):
        assert st["exact_fraction"] == 1.0, st
    # a fresh index over the exported lists answers identically (the slack layout is invisible)
    fresh = gpu.HipIndexIVFFlat(cen, off, ids, codes, 8)
    fresh.form = form
    D2, I2 = fresh.search(xq, 10)
    assert np.array_equal(I, I2) and np.array_equal(D, D2)


def test_ivf_append_rescales_fp16_image(gpu, oracle):
    """An append whose rows leave the fp16 image's scale (max|x| past 2^e of the build) drops the image; the next
    search rebuilds it at the new scale and stays exact against the oracle."""
    rng = np.random.default_rng(12)
    d, nlist = 32, 16
    xb = rng.uniform(-1, 1, (6000, d)).astype(np.float32)
    xb[5000:] *= np.float32(40.0)
    xq = np.concatenate([xb[5000:5020] + np.float32(1e-2), rng.uniform(-1, 1, (20, d)).astype(np.float32)])
    cen = np.ascontiguousarray(xb[:nlist * 100:100])
    off0, ids0, codes0 = build_ivf_lists(xb[:5000], cen)
    ix = gpu.HipIndexIVFFlat(cen, off0, ids0, codes0, 4)
    ix.search(xq, 10)
    ix.add(xb[5000:])
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == ix.FORM_HALF_EXACT
    off, ids, codes = build_ivf_lists(xb, cen)
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 4)
    st = check_topk_parity(xb, xq, D, I, Do, Io)
    assert st["exact_fraction"] == 1.0, st


@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_nan_and_overflow_queries_pad_like_faiss(gpu, oracle, metric):
    """on the IVF exact form a NaN query (and, for L2, an overflowing one) returns FAISS's all −1 labels
    (its heap admits neither NaN nor +inf); the batch's other queries keep exact parity."""
    rng = np.random.default_rng(8 + metric)
    xb = rng.standard_normal((20_000, 48), dtype=np.float32)
    xq = rng.standard_normal((40, 48), dtype=np.float32)
    xq[3, 0] = np.nan
    bad = [3]
    if metric == 0:
        xq[4] = np.float32(3e38)
        bad.append(4)
    cen = np.ascontiguousarray(xb[::500][:40])
    off, ids, codes = build_ivf_lists(xb, cen, metric)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, codes, 6, metric=metric)
    D, I = ix.search(xq, 10)
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 6, metric)
    for b in bad:
        assert (Io[b] == -1).all()
        assert (I[b] == -1).all(), (b, I[b])
    good = np.array([i for i in range(len(xq)) if i not in bad])
    st = check_topk_parity(xb, xq[good], D[good], I[good], Do[good], Io[good], metric)
    assert st["exact_fraction"] == 1.0, st


@pytest.mark.parametrize("form", [6, 5, 0, 7])
def test_ivf_empty_l2_index_then_append(gpu, oracle, form):
    """an L2 IVF index created with zero rows has no norm array (compute_row_norms skips n = 0);
    the first append's relayout must give it one, because ivf_append_rows writes the new rows' norms into it and the
    decomposed / fp16 scans read them.  After the append every exact form's ids equal the oracle's IndexIVFFlat."""
    rng = np.random.default_rng(31 + form)
    d, nlist = 48, 16
    xb = rng.standard_normal((6000, d), dtype=np.float32)
    xq = rng.standard_normal((64, d), dtype=np.float32)
    cen = np.ascontiguousarray(xb[:nlist * 100:100])
    ix = gpu.HipIndexIVFFlat(cen, np.zeros(nlist + 1, np.int64), np.zeros(0, np.int64),
                             np.zeros((0, d), np.float32), 4)
    ix.form = form
    D, I = ix.search(xq[:2], 5)
    assert (I == -1).all()
    ix.add(xb[:3000])
    ix.add(xb[3000:])
    assert ix.ntotal == len(xb)
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == form
    off, ids, codes = build_ivf_lists(xb, cen)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 4)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    st = check_topk_parity(xb, xq, D, I, Do, Io)
    if form in (5, 6, 7):
        assert st["exact_fraction"] == 1.0, st


@pytest.mark.parametrize("form", [5, 0, 7])
def test_ivf_search_probes_device_reused_buffer(gpu, oracle, form):
    """search_probes_device (caller-supplied probe lists, no coarse step) must compute ‖q‖² of
    THIS call's queries: two calls on one device buffer whose contents change in between (same pointer, same nq)
    each equal the oracle's search of their own queries."""
    import torch
    rng = np.random.default_rng(77)
    d, nlist, nprobe, nq = 64, 32, 6, 48
    xb = rng.standard_normal((12000, d), dtype=np.float32)
    cen = np.ascontiguousarray(xb[:nlist * 300:300])
    off, ids, codes = build_ivf_lists(xb, cen)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, codes, nprobe)
    ix.form = form
    dev = torch.device("cuda", 0)
    q_t = torch.empty((nq, d), device=dev, dtype=torch.float32)
    p_t = torch.empty((nq, nprobe), device=dev, dtype=torch.int64)
    Dt = torch.empty((nq, 10), device=dev)
    It = torch.empty((nq, 10), device=dev, dtype=torch.int64)
    stream = torch.cuda.current_stream().cuda_stream
    for rep in range(2):
        xq = (rng.standard_normal((nq, d)) * (1.0 + 3.0 * rep)).astype(np.float32)
        q_t.copy_(torch.from_numpy(xq))
        Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, nprobe)
        p_t.copy_(torch.from_numpy(Po))
        if rep == 0:  # a full search on the same buffer first: the quantizer caches ‖q‖² of this pointer
            ix.search_device(nq, q_t.data_ptr(), 10, Dt.data_ptr(), It.data_ptr(), stream)
        ix.search_probes_device(nq, q_t.data_ptr(), p_t.data_ptr(), 10, Dt.data_ptr(), It.data_ptr(), stream)
        torch.cuda.synchronize()
        D, I = Dt.cpu().numpy(), It.cpu().numpy()
        st = check_topk_parity(xb, xq, D, I, Do, Io)
        if form in (5, 7):
            assert st["exact_fraction"] == 1.0, (rep, st)


def test_peer_access_query_multi_device_handles(gpu, oracle):
    """a multi-device handle enables peer access between every shard's device and the first
    shard's at create (hipann_peer_access).  On the one-GPU box every shard sits on device 0: the state is "same
    device" (not applicable) for each, and searches still equal the oracle.  With >= 2 devices visible the pair
    must report enabled where hipDeviceCanAccessPeer allows it."""
    import torch
    xb, xq = faiss_metal_case(6000, 24, 32)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 16, 4, devices=[0, 0, 0])
    assert ix.peer_access() == [ix.PEER_SAME_DEVICE] * 3
    D, I = ix.search(xq, 10)
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 4)
    check_topk_parity(xb, xq, D, I, Do, Io)
    fx = gpu.HipIndexFlat(32, 0, xb, devices=[0, 0])
    assert fx.peer_access() == [fx.PEER_SAME_DEVICE] * 2
    single = gpu.HipIndexFlat(32, 0, xb)
    assert single.peer_access() == [single.PEER_SAME_DEVICE]
    if torch.cuda.device_count() >= 2:
        two = gpu.HipIndexFlat(32, 0, xb, devices=[0, 1])
        can = torch.cuda.can_device_access_peer(0, 1) and torch.cuda.can_device_access_peer(1, 0)
        assert two.peer_access() == [two.PEER_SAME_DEVICE, two.PEER_ENABLED if can else two.PEER_UNAVAILABLE]


@pytest.mark.parametrize("metric", [0, 1])
def test_ivf_i8_form_nonfinite_and_scaled(gpu, oracle, metric):
    """Form 7 (the int8 image, one scale per row): rows at very different magnitudes (each row has its own scale, so
    small rows keep their relative precision), a NaN query (FAISS's all −1 labels) and an append (the image is released and rebuilt at
    the next search); ids equal the oracle's throughout."""
    rng = np.random.default_rng(70 + metric)
    d = 80
    xb = rng.standard_normal((12_000, d), dtype=np.float32)
    xb[::3] *= np.float32(1e-3)
    xb[1::7] *= np.float32(50.0)
    xq = rng.standard_normal((60, d), dtype=np.float32)
    xq[5, 7] = np.nan
    cen = np.ascontiguousarray(xb[::400][:30])
    off, ids, codes = build_ivf_lists(xb, cen, metric)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, codes, 5, metric=metric)
    ix.form = 7
    D, I = ix.search(xq, 10)
    assert ix.last_search_path()["form"] == 7
    Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 5, metric)
    assert (Io[5] == -1).all() and (I[5] == -1).all()
    good = np.array([i for i in range(len(xq)) if i != 5])
    st = check_topk_parity(xb, xq[good], D[good], I[good], Do[good], Io[good], metric)
    assert st["exact_fraction"] == 1.0, st
    # an append releases the int8 image; the next search rebuilds it over the grown lists
    xa = (rng.standard_normal((3000, d)) * 3.0).astype(np.float32)
    ix.add(xa)
    xall = np.concatenate([xb, xa])
    off2, ids2, codes2 = build_ivf_lists(xall, cen, metric)
    D2, I2 = ix.search(xq[good], 10)
    assert ix.last_search_path()["form"] == 7
    Do2, Io2, _ = oracle.ivf_search(cen, off2, ids2, codes2, xq[good], 10, 5, metric)
    st = check_topk_parity(xall, xq[good], D2, I2, Do2, Io2, metric)
    assert st["exact_fraction"] == 1.0, st
