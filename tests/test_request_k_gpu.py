"""request_k above 12 on the exact forms.

The extension asks the GPU index for request_k = min(k + |tombstones|, ntotal) rows (src/faiss_index.cpp:713-715):
with k = 10 and 20 deleted rows that is 30.  Until r03 the exact forms (Flat form 4, IVF forms 5/6) served
request_k <= 12 only and everything larger fell to the 3-term split scans (6 bf16 products per element).  Now:

* Flat form 4, bounded passes: the filter keeps kf = min(64, max(32, 2·kout)) candidates per query; any kout <= kf
  stays exact (queries the first rerank cannot certify go to the all-candidate rerank, certified against the
  pass bound).  The LDS list kernels (small tables, small batches) hold kf up to their LDS budget and need
  kf >= kout + 4.
* IVF forms 5/6: the scans write every wave's 16-list as a sub-list of the slot; the rerank filters
  kf = min(64, max(kout + 4, 2·kout)) candidates and certifies against both its kf-th key and the smallest full
  sub-list's 16th key (qbound) — kout <= 60.

Every case is checked against the oracle (FAISS IndexFlat / IndexIVFFlat restatements) with the parity rule, and
the path that ran is read back (hipann_last_search_path) so a silent fall to the split scans would fail.
"""
from __future__ import annotations

import numpy as np
import pytest

from _data import build_ivf_lists, check_topk_parity, faiss_metal_case

pytestmark = pytest.mark.gpu


def _flat_kf(k):
    return 32 if k <= 12 else min(64, max(32, 2 * k))


def _ivf_kf(k):
    return 16 if k <= 12 else min(64, max(k + 4, 2 * k))


@pytest.mark.parametrize("form", [4, 5])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [13, 20, 30, 32, 64])
def test_flat_bounded_passes_request_k(gpu, oracle, metric, k, form):
    """Flat form 4 through the bounded passes (600k x 64 rows >= the 512K-row seed threshold, nq 256): exact at
    request_k 13-64, ids as the fp32 form's except in near-tie windows, the oracle's parity rule on 48 queries."""
    rng = np.random.default_rng(100 + k + metric)
    n, d, nq = 600_000, 64, 256
    xb = rng.standard_normal((n, d), dtype=np.float32)
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    ix = gpu.HipIndexFlat(d, metric, xb)
    ix.form = form
    D, I = ix.search(xq, k)
    path = ix.last_search_path()
    assert path["form"] == form and path["filter_k"] == (_flat_kf(k) if form == 4 else 64), path
    assert ix.rerank_fallbacks() <= nq // 16, ix.rerank_fallbacks()
    Do, Io = oracle.flat_search(xb, xq[:48], k, metric)
    check_topk_parity(xb, xq[:48], D[:48], I[:48], Do, Io, metric)
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, k)
    assert (I == I0).mean() >= 0.995
    scale = np.sum(xq.astype(np.float64) ** 2, 1)[:, None] + np.max(np.sum(xb.astype(np.float64) ** 2, 1))
    assert (np.abs(D - D0) <= 1e-5 * scale).all()
    ix.close()


@pytest.mark.parametrize("k", [13, 20, 28, 32, 64])
@pytest.mark.parametrize("nq", [64, 300])
def test_flat_list_kernels_request_k(gpu, oracle, k, nq):
    """Flat form 4 on the LDS-list kernel (20k rows: below the bounded passes' threshold): exact while the
    list holds kf >= k + 4, else the 3-term split; either way the oracle's parity rule."""
    xb, xq = faiss_metal_case(20000, nq, 128)
    ix = gpu.HipIndexFlat(128, 0, xb)
    D, I = ix.search(xq, k)
    Do, Io = oracle.flat_search(xb, xq, k, 0)
    check_topk_parity(xb, xq, D, I, Do, Io, 0)
    path = ix.last_search_path()
    if path["filter_k"]:
        assert path["form"] == ix.FORM_BF16_EXACT and path["filter_k"] >= k + 4, path
    else:  # the 3-term split, or the fp32 matrix cores where its LDS lists are too short (k > 38)
        assert path["form"] in (ix.FORM_SPLIT3, ix.FORM_FP32), path
    if k <= 28:  # the list holds >= 32 at every block shape: exact
        assert path["filter_k"] >= k + 4, path
    ix.close()


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [20, 32])
def test_flat_bounded_passes_request_k_near_duplicates(gpu, oracle, metric, k):
    """The near-duplicate fixture of test_flat_bf16_flagged_queries_candidate_rerank at request_k 20 / 32:
    16K base rows x 40 copies + 1e-4 noise (640k x 64, nq 256) — the first rerank cannot certify the queries,
    the all-candidate rerank does; ids follow the oracle's parity rule on every query."""
    rng = np.random.default_rng(31 + k + metric)
    base = rng.standard_normal((16_000, 64), dtype=np.float32)
    xb = np.repeat(base, 40, axis=0)
    xb += 1e-4 * rng.standard_normal(xb.shape, dtype=np.float32)
    xb = xb[rng.permutation(len(xb))]
    xq = rng.standard_normal((256, 64), dtype=np.float32)
    ix = gpu.HipIndexFlat(64, metric, xb)
    D, I = ix.search(xq, k)
    path = ix.last_search_path()  # the default int8 filter is 64 deep; form 4's follows k
    assert path["filter_k"] == (64 if path["form"] == ix.FORM_I8_EXACT else _flat_kf(k)), path
    Do, Io = oracle.flat_search(xb, xq, k, metric)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    assert ix.rerank_fallbacks() < len(xq) // 4, ix.rerank_fallbacks()
    ix.close()


def _ivf(gpu, xb, nlist, nprobe, metric=0):
    cen = np.ascontiguousarray(xb[:: len(xb) // nlist][:nlist])
    off, ids, codes = build_ivf_lists(xb, cen, metric)
    return gpu.HipIndexIVFFlat(cen, off, ids, codes, nprobe, metric), (cen, off, ids, codes)


@pytest.mark.parametrize("form", [5, 6])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("k", [13, 20, 30, 32, 60, 64])
def test_ivf_exact_forms_request_k(gpu, oracle, form, metric, k):
    """IVF forms 5 / 6 at request_k 13-60 (sub-list slots + a kf-deep rerank; 64: the 3-term scan): probe
    lists equal the oracle's, ids follow the parity rule, distances are the direct fp32 form."""
    xb, xq = faiss_metal_case(20000, 96, 96)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 64, 8, metric)
    ix.form = form
    D, I = ix.search(xq, k)
    path = ix.last_search_path()
    if k <= 60:
        assert path == {"form": form, "filter_k": _ivf_kf(k), "sublists": 8}, path
    else:
        # the 3-term scan keeps 16-lists, so k = 64 takes the VALU decomposed scan (exact fp32 products)
        assert path["filter_k"] == 0 and path["form"] == ix.FORM_DECOMPOSED_VALU, path
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, k, 8, metric)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(xb, xq, D, I, Do, Io, metric)
    if k <= 60:
        v = I >= 0
        assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)
    ix.close()


@pytest.mark.parametrize("form", [5, 6])
@pytest.mark.parametrize("k", [13, 20, 40])
def test_ivf_request_k_exact_ties_scan_order(gpu, oracle, form, k):
    """Exact ties at request_k > 12: every vector stored 3 times in its list (copies in different row orders,
    scattered labels), so distances tie in threes across the 20th/40th rank.  The rerank (or the device
    fallback for the queries it cannot certify) applies FAISS's scan-order admission: slot for slot equal to the
    oracle (reference edge case: duplicates, test/sql/edge_cases.test:75-83)."""
    base, xq = faiss_metal_case(3000, 120, 64)
    cen = np.ascontiguousarray(base[::150][:20])
    off0, ids0, codes0 = build_ivf_lists(base, cen, 0)
    rng = np.random.default_rng(9 + k)
    off = off0 * 3
    codes = np.ascontiguousarray(np.concatenate([np.concatenate([codes0[off0[l]:off0[l + 1]],
                                                                 codes0[off0[l]:off0[l + 1]][::-1],
                                                                 codes0[off0[l]:off0[l + 1]]]) for l in range(len(cen))]))
    labels = rng.permutation(len(codes)).astype(np.int64) * 3 + 11
    ix = gpu.HipIndexIVFFlat(cen, off, labels, codes, 5, 0)
    ix.form = form
    D, I = ix.search(xq, k)
    assert ix.last_search_path()["sublists"] == 8
    Do, Io, Po = oracle.ivf_search(cen, off, labels, codes, xq, k, 5, 0)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    assert np.array_equal(I, Io), f"{(I != Io).any(axis=1).sum()} queries differ"
    v = I >= 0
    assert np.allclose(D[v], Do[v], rtol=2e-6, atol=1e-6)
    ix.close()


def test_ivf_request_k_long_lists_many_chunks(gpu, oracle):
    """Sub-list slots on lists of several 2048-row chunks and several query groups (the slot index times the
    sub-list count), nq 70, request_k 25."""
    xb, xq = faiss_metal_case(21000, 70, 64)
    ix, (cen, off, ids, codes) = _ivf(gpu, xb, 4, 2)
    assert np.diff(off).max() > 2048
    D, I = ix.search(xq, 25)
    assert ix.last_search_path()["sublists"] == 8
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 25, 2, 0)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(xb, xq, D, I, Do, Io)
    ix.close()
