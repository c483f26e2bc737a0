"""ctypes wrapper of oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker (or the timed CPU baseline).  The product path (duckdb-annsearch_amd/hipann.py →
libhipann.so) never imports it.  See oracle.c for the reference file:line each function restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"

L2, IP = 0, 1

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = C.CDLL(str(LIB_PATH))
        f, i64, i32, u32 = C.POINTER(C.c_float), C.POINTER(C.c_int64), C.c_int, C.POINTER(C.c_uint32)
        u8, d64 = C.POINTER(C.c_uint8), C.POINTER(C.c_double)
        _lib.oracle_flat_search.argtypes = [f, C.c_int64, i32, f, C.c_int64, i32, i32, C.c_int64, f, i64]
        _lib.oracle_ivf_search.argtypes = [f, i32, i64, i64, f, i32, f, C.c_int64, i32, i32, i32, f, i64, i64]
        _lib.oracle_ivf_search_preassigned.argtypes = [i64, i64, f, i32, f, C.c_int64, i32, i32, i64, i32, f, i64]
        _lib.oracle_exact_dists.argtypes = [f, i32, f, i64, C.c_int64, i32, d64]
        _lib.oracle_batch_distances.argtypes = [f, f, i32, i32, i32, f]
        _lib.oracle_batch_distances_simd.argtypes = [f, f, i32, i32, i32, f]
        _lib.oracle_multi_batch_distances.argtypes = [f, f, u32, i32, i32, i32, f]
        _lib.oracle_sq8_train.argtypes = [f, C.c_int64, i32, f, f]
        _lib.oracle_sq8_encode.argtypes = [f, C.c_int64, i32, f, f, u8]
        _lib.oracle_sq8_decode.argtypes = [u8, C.c_int64, i32, f, f, f]
        _lib.oracle_sq8_distances_ids.argtypes = [f, u8, f, f, i32, u32, u32, i32, i32, f]
        _lib.oracle_diskann_search_batch.argtypes = [f, u8, f, f, C.c_uint32, i32, u32, i32, u32, i32, f, i32, i32,
                                                     i32, i32, i64, f, i64]
        _lib.oracle_num_threads.restype = C.c_int
        _lib.oracle_kmeans_train.argtypes = [f, C.c_int64, i32, i32, i32, C.c_int64, i32, C.c_uint64, i32, f, i64]
        _lib.oracle_kmeans_train.restype = C.c_int
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def num_threads() -> int:
    return lib().oracle_num_threads()


def flat_search(xb, xq, k, metric=L2, label_offset=0):
    """FAISS IndexFlat{L2,IP}::search restated (see oracle.c).  Pads are (±FLT_MAX, -1)."""
    xb, xq = _f32(xb), _f32(xq)
    n, d = xb.shape if xb.ndim == 2 else (0, xq.shape[1])
    nq = xq.shape[0]
    D = np.empty((nq, k), np.float32)
    I = np.empty((nq, k), np.int64)
    lib().oracle_flat_search(_p(xb, C.c_float), n, d, _p(xq, C.c_float), nq, k, metric, label_offset,
                             _p(D, C.c_float), _p(I, C.c_int64))
    return D, I


def ivf_search(centroids, list_off, ids, codes, xq, k, nprobe, metric=L2):
    """FAISS IndexIVFFlat::search restated; returns (D, I, probes)."""
    centroids, codes, xq = _f32(centroids), _f32(codes), _f32(xq)
    list_off = np.ascontiguousarray(list_off, np.int64)
    ids = np.ascontiguousarray(ids, np.int64)
    nlist, d = centroids.shape
    nq = xq.shape[0]
    npr = min(nprobe, nlist)
    D = np.empty((nq, k), np.float32)
    I = np.empty((nq, k), np.int64)
    P = np.empty((nq, npr), np.int64)
    lib().oracle_ivf_search(_p(centroids, C.c_float), nlist, _p(list_off, C.c_int64), _p(ids, C.c_int64),
                            _p(codes, C.c_float), d, _p(xq, C.c_float), nq, k, nprobe, metric,
                            _p(D, C.c_float), _p(I, C.c_int64), _p(P, C.c_int64))
    return D, I, P


def ivf_search_preassigned(list_off, ids, codes, xq, k, probes, metric=L2):
    """FAISS IndexIVF::search_preassigned restated: the lists of `probes` (nq x nprobe, probe order) scanned in the
    direct form — the IVF scan of a given probe list (tests hold the GPU scan to it on the GPU's own probe lists)."""
    codes, xq = _f32(codes), _f32(xq)
    list_off = np.ascontiguousarray(list_off, np.int64)
    ids = np.ascontiguousarray(ids, np.int64)
    probes = np.ascontiguousarray(probes, np.int64)
    nq, npr = probes.shape
    d = xq.shape[1]
    D = np.empty((nq, k), np.float32)
    I = np.empty((nq, k), np.int64)
    lib().oracle_ivf_search_preassigned(_p(list_off, C.c_int64), _p(ids, C.c_int64), _p(codes, C.c_float), d,
                                        _p(xq, C.c_float), nq, k, npr, _p(probes, C.c_int64), metric,
                                        _p(D, C.c_float), _p(I, C.c_int64))
    return D, I


def exact_dists(xb, q, labels, metric=L2):
    """fp64 distance of query q to rows `labels` of xb (NaN for labels < 0)."""
    xb, q = _f32(xb), _f32(q)
    labels = np.ascontiguousarray(labels, np.int64)
    out = np.empty(labels.shape, np.float64)
    lib().oracle_exact_dists(_p(xb, C.c_float), xb.shape[1], _p(q, C.c_float), _p(labels, C.c_int64), labels.size,
                             metric, _p(out, C.c_double))
    return out


def batch_distances(query, cands, metric=L2):
    query, cands = _f32(query), _f32(cands)
    n, d = cands.shape
    out = np.empty(n, np.float32)
    lib().oracle_batch_distances(_p(query, C.c_float), _p(cands, C.c_float), n, d, metric, _p(out, C.c_float))
    return out


def multi_batch_distances(queries, cands, qmap, metric=L2):
    queries, cands = _f32(queries), _f32(cands)
    qmap = np.ascontiguousarray(qmap, np.uint32)
    n, d = cands.shape
    out = np.empty(n, np.float32)
    lib().oracle_multi_batch_distances(_p(queries, C.c_float), _p(cands, C.c_float), _p(qmap, C.c_uint32), n, d,
                                       metric, _p(out, C.c_float))
    return out


def sq8_train(x):
    x = _f32(x)
    n, d = x.shape
    mins = np.empty(d, np.float32)
    scale = np.empty(d, np.float32)
    lib().oracle_sq8_train(_p(x, C.c_float), n, d, _p(mins, C.c_float), _p(scale, C.c_float))
    return mins, scale


def sq8_encode(x, mins, scale):
    x, mins, scale = _f32(x), _f32(mins), _f32(scale)
    n, d = x.shape
    codes = np.empty((n, d), np.uint8)
    lib().oracle_sq8_encode(_p(x, C.c_float), n, d, _p(mins, C.c_float), _p(scale, C.c_float),
                            _p(codes, C.c_uint8))
    return codes


def sq8_decode(codes, mins, scale):
    codes = np.ascontiguousarray(codes, np.uint8)
    mins, scale = _f32(mins), _f32(scale)
    n, d = codes.shape
    out = np.empty((n, d), np.float32)
    lib().oracle_sq8_decode(_p(codes, C.c_uint8), n, d, _p(mins, C.c_float), _p(scale, C.c_float),
                            _p(out, C.c_float))
    return out


def sq8_distances_ids(queries, codes, mins, scale, ids, qmap, metric=L2):
    queries, mins, scale = _f32(queries), _f32(mins), _f32(scale)
    codes = np.ascontiguousarray(codes, np.uint8)
    ids = np.ascontiguousarray(ids, np.uint32)
    qmap = np.ascontiguousarray(qmap, np.uint32)
    out = np.empty(ids.size, np.float32)
    lib().oracle_sq8_distances_ids(_p(queries, C.c_float), _p(codes, C.c_uint8), _p(mins, C.c_float),
                                   _p(scale, C.c_float), codes.shape[1], _p(ids, C.c_uint32), _p(qmap, C.c_uint32),
                                   ids.size, metric, _p(out, C.c_float))
    return out


def diskann_search_batch(adj, entry_points, queries, k, l_search, metric=L2, vecs=None, codes=None, mins=None,
                         scale=None):
    """DiskProvider::search_batch restated.  Returns (ids[nq,k] int64, dists[nq,k], stats{evals,steps})."""
    queries = _f32(queries)
    adj = np.ascontiguousarray(adj, np.uint32)
    eps = np.ascontiguousarray(entry_points, np.uint32)
    N, R = adj.shape
    nq, d = queries.shape
    kk = min(k, N)
    out_i = np.empty((nq, kk), np.int64)
    out_d = np.empty((nq, kk), np.float32)
    stats = np.zeros(2, np.int64)
    if codes is not None:
        codes = np.ascontiguousarray(codes, np.uint8)
        mins, scale = _f32(mins), _f32(scale)
        vp = None
    else:
        vecs = _f32(vecs)
        vp = vecs
    lib().oracle_diskann_search_batch(_p(vp, C.c_float), _p(codes, C.c_uint8), _p(mins, C.c_float),
                                      _p(scale, C.c_float), N, d, _p(adj, C.c_uint32), R, _p(eps, C.c_uint32),
                                      eps.size, _p(queries, C.c_float), nq, kk, l_search, metric,
                                      _p(out_i, C.c_int64), _p(out_d, C.c_float), _p(stats, C.c_int64))
    return out_i, out_d, {"evals": int(stats[0]), "steps": int(stats[1])}


def kmeans_train(x, nlist, metric=L2, train_sample=0, niter=25, seed=1234, init=1):
    """oracle_kmeans_train: the restatement of hipann_ivf_train (stride sample, subsample, init, Lloyd with
    FAISS's split_clusters / spherical renorm).  Returns (centroids nlist x d, last iteration's cluster sizes)."""
    x = _f32(x)
    n, d = x.shape
    cen = np.empty((nlist, d), np.float32)
    sizes = np.empty(nlist, np.int64)
    rc = lib().oracle_kmeans_train(_p(x, C.c_float), n, d, metric, nlist, train_sample, niter, seed, init,
                                   _p(cen, C.c_float), _p(sizes, C.c_int64))
    if rc != 0:
        raise ValueError("oracle_kmeans_train: bad arguments (n < nlist?)")
    return cen, sizes
