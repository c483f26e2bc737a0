"""CPU baseline legs for bench.py — TEST / MEASUREMENT INFRASTRUCTURE ONLY (never on the product path).

The reference's CPU path for the FAISS configurations is FAISS 1.13.2's CPU index (absent here and on
the GPU box).  These functions restate the part of it that dominates the time, at the speed class of
the original:

* ``flat_blas_qps`` — IndexFlatL2::search for nq >= 20 (knn_L2sqr → exhaustive_L2sqr_blas): query and
  database norms, then 4096 × 1024 (query × database) blocks of ``x·yᵀ`` through a CPU BLAS sgemm
  (torch CPU → MKL/OpenBLAS, all host threads), ``‖x‖² + ‖y‖² − 2·ip`` clamped at 0, and a running
  top-k per query.  Timed on a bounded slice of the database, reported as queries/s on the full one.
* ``ivf_qps`` — IndexIVFFlat::search: the C oracle (oracle.c, OpenMP over queries, SIMD direct
  distances, FAISS heaps) on a bounded subset of the query batch.
"""
from __future__ import annotations

import os
import time

import numpy as np


def flat_blas_qps(xb_slice: np.ndarray, xq: np.ndarray, k: int, n_full: int, metric: int = 0, threads: int = 0):
    """Time the BLAS-path restatement over ``xb_slice`` (rows of the full database) for all of ``xq``;
    return (queries/s extrapolated to n_full rows, seconds, threads)."""
    import torch

    if threads:
        torch.set_num_threads(threads)
    nth = torch.get_num_threads()
    xq_t = torch.from_numpy(np.ascontiguousarray(xq, np.float32))
    xb_t = torch.from_numpy(np.ascontiguousarray(xb_slice, np.float32))
    nq, n = xq_t.shape[0], xb_t.shape[0]
    t0 = time.perf_counter()
    qn = (xq_t * xq_t).sum(1) if metric == 0 else None
    best_d = torch.full((nq, k), float("inf"))
    best_i = torch.full((nq, k), -1, dtype=torch.int64)
    for j0 in range(0, n, 1024):
        xb_blk = xb_t[j0:j0 + 1024]
        yn = (xb_blk * xb_blk).sum(1) if metric == 0 else None
        for i0 in range(0, nq, 4096):
            ip = xq_t[i0:i0 + 4096] @ xb_blk.T
            if metric == 0:
                dis = (qn[i0:i0 + 4096, None] + yn[None, :] - 2 * ip).clamp_min_(0)
            else:
                dis = -ip
            ids = torch.arange(j0, j0 + xb_blk.shape[0]).expand(dis.shape[0], -1)
            cat_d = torch.cat([best_d[i0:i0 + 4096], dis], 1)
            cat_i = torch.cat([best_i[i0:i0 + 4096], ids], 1)
            v, p = torch.topk(cat_d, k, dim=1, largest=False, sorted=True)
            best_d[i0:i0 + 4096] = v
            best_i[i0:i0 + 4096] = torch.gather(cat_i, 1, p)
    dt = time.perf_counter() - t0
    seconds_full = dt * (n_full / n)
    return nq / seconds_full, dt, nth


def ivf_qps(centroids, list_off, ids, codes, xq, k: int, nprobe: int, metric: int = 0):
    """Time the C oracle's IndexIVFFlat::search on ``xq``; return (queries/s, seconds, threads)."""
    qps, dt, nth, _, _ = ivf_search_timed(centroids, list_off, ids, codes, xq, k, nprobe, metric)
    return qps, dt, nth


def ivf_search_timed(centroids, list_off, ids, codes, xq, k: int, nprobe: int, metric: int = 0):
    """ivf_qps plus the CPU path's answers (D, I) for those queries — bench.py compares them with the GPU ids
    (oracle/parity.py).  Returns (queries/s, seconds, threads, D, I)."""
    from . import oracle as O

    t0 = time.perf_counter()
    D, I, _ = O.ivf_search(centroids, list_off, ids, codes, xq, k, nprobe, metric)
    dt = time.perf_counter() - t0
    return xq.shape[0] / dt, dt, O.num_threads(), D, I
