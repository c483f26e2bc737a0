"""ivf_build — build an IVFFlat shard on the GPU for the benchmark / integration tests.

The extension builds its IVF index on the CPU with FAISS (faiss_index.cpp:302-332: train on a
stride sample, then add) and copies it to the GPU (index_cpu_to_metal_ivf,
MetalIndexIVFFlat.mm:283-326).  FAISS is absent here, so this module does the same work on the GPU
(SURVEY §8f rank 4): k-means over a 256·nlist-point sample (FAISS's default max_points_per_centroid,
25 iterations, seeded init from the sample), assignment of every row with the Flat kernels (k = 1),
a stable counting sort into list-contiguous storage, and hipann_ivf_create_device on the result.

Multi-GPU: rank 0 trains and broadcasts the centroids; every rank assigns and stores only its own
rows (its lists' rows come from its shard of the database), so list l is split across ranks by row
range — equivalent to sharding the lists' contents, and every rank scans only its local rows.
"""
from __future__ import annotations

import numpy as np


def kmeans_pp_init(torch, x, nlist: int, g):
    """k-means++ seeding (D² sampling).  FAISS seeds with a random sample; on well-separated clusters in
    high dimension that start leaves averaged centroids that absorb neighbouring clusters (lists of 10×
    the mean), so the build uses D² seeding instead (IVF build)."""
    m = x.shape[0]
    xn = (x * x).sum(1)
    first = int(torch.randint(0, m, (1,), generator=g))
    cen = [x[first]]
    d2 = (xn - 2 * (x @ x[first]) + xn[first]).clamp_min_(0)
    u = torch.rand((nlist,), generator=g).to(x.device)
    for i in range(1, nlist):
        cdf = torch.cumsum(d2, 0)
        idx = int(torch.searchsorted(cdf, u[i] * cdf[-1]).clamp_max(m - 1))
        c = x[idx]
        cen.append(c)
        d2 = torch.minimum(d2, (xn - 2 * (x @ c) + xn[idx]).clamp_min_(0))
    return torch.stack(cen).contiguous()


def kmeans(torch, hipann, x, nlist: int, niter: int = 25, seed: int = 1234, metric: int = 0, init: str = "kmeans++"):
    """Lloyd k-means on the GPU (assignment through the Flat kernels).  x: (m, d) CUDA fp32."""
    m, d = x.shape
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    if init == "kmeans++":
        cen = kmeans_pp_init(torch, x, nlist, g)
    else:
        perm = torch.randperm(m, generator=g)[:nlist].to(x.device)
        cen = x[perm].clone()
    stream = torch.cuda.current_stream().cuda_stream
    D = torch.empty((m, 1), device=x.device, dtype=torch.float32)
    I = torch.empty((m, 1), device=x.device, dtype=torch.int64)
    for _ in range(niter):
        idx = hipann.HipIndexFlatDevice(d, 0, cen.data_ptr(), nlist, x.device.index, copy=False)
        idx.search_device(m, x.data_ptr(), 1, D.data_ptr(), I.data_ptr(), stream)
        torch.cuda.synchronize()
        idx.close()
        a = I[:, 0]
        counts = torch.bincount(a, minlength=nlist).to(torch.float32)
        sums = torch.zeros_like(cen).index_add_(0, a, x)
        new = sums / counts.clamp_min(1)[:, None]
        empty = counts == 0
        if bool(empty.any()):  # FAISS splits big clusters; here: re-seed from random sample points
            ne = int(empty.sum())
            pick = torch.randint(0, m, (ne,), generator=g).to(x.device)
            new[empty] = x[pick]
        cen = new.contiguous()
    return cen


def build_ivf_shard(torch, hipann, xb, row0: int, n_total: int, nlist: int, nprobe: int, metric: int, rank: int,
                    world: int, centres_seed: int = 1234, train_points_per_list: int = 256):
    """Returns (HipIndexIVFFlat over this rank's rows, info dict)."""
    import torch.distributed as dist

    dev = xb.device
    n_local, d = xb.shape
    # ---- train (rank 0) ----
    if rank == 0:
        m = min(n_local, train_points_per_list * nlist)
        stride = max(1, n_local // m)
        sample = xb[::stride][:m].contiguous()
        cen = kmeans(torch, hipann, sample, nlist, seed=centres_seed)
        del sample
    else:
        cen = torch.empty((nlist, d), device=dev, dtype=torch.float32)
    if world > 1:
        dist.broadcast(cen, 0)
    cen = cen.contiguous()
    # ---- assign (Flat kernels, k = 1, chunks of 1M rows) ----
    stream = torch.cuda.current_stream().cuda_stream
    assign = torch.empty((n_local,), device=dev, dtype=torch.int64)
    qidx = hipann.HipIndexFlatDevice(d, metric, cen.data_ptr(), nlist, dev.index, copy=False)
    chunk = 1_000_000
    Dc = torch.empty((chunk, 1), device=dev, dtype=torch.float32)
    Ic = torch.empty((chunk, 1), device=dev, dtype=torch.int64)
    for s in range(0, n_local, chunk):
        e = min(n_local, s + chunk)
        qidx.search_device(e - s, xb[s:e].data_ptr(), 1, Dc.data_ptr(), Ic.data_ptr(), stream)
        assign[s:e].copy_(Ic[:e - s, 0])
    torch.cuda.synchronize()
    qidx.close()
    del Dc, Ic
    # ---- list-contiguous storage (stable counting sort) ----
    order = torch.sort(assign, stable=True).indices
    counts = torch.bincount(assign, minlength=nlist)
    offsets = np.zeros(nlist + 1, np.int64)
    offsets[1:] = np.cumsum(counts.cpu().numpy())
    codes = torch.empty_like(xb)
    for s in range(0, n_local, chunk):
        e = min(n_local, s + chunk)
        codes[s:e] = xb[order[s:e]]
    ids = (order + row0).contiguous()
    del order, assign
    index = hipann.HipIndexIVFFlat.from_device(d, metric, nlist, nprobe, cen.data_ptr(), offsets, ids.data_ptr(),
                                               codes.data_ptr(), dev.index, copy=False)
    index._keep = (cen, codes, ids)  # borrowed by the library
    index._offsets = offsets
    sizes = np.diff(offsets)
    info = {"nlist": nlist, "nprobe": nprobe, "list_size_min": int(sizes.min()), "list_size_max": int(sizes.max()),
            "list_size_mean": float(sizes.mean())}
    return index, info


def scan_bytes(index, probes: np.ndarray, d: int) -> float:
    """Algorithmic HBM bytes of one batch's list scan on this shard: every distinct probed list read
    once, |l|·(4d + 8) bytes (codes + label)."""
    sizes = np.diff(index._offsets)
    distinct = np.unique(probes[probes >= 0])
    return float(sizes[distinct].sum()) * (4 * d + 8)


def scan_pairs(index, probes: np.ndarray) -> int:
    """(query, row) distance evaluations of one batch on this shard: Σ_q Σ_p |l(q, p)|."""
    sizes = np.diff(index._offsets)
    p = probes[probes >= 0]
    return int(sizes[p].sum())


def scan_group_rows(index, probes: np.ndarray, group: int = 32) -> int:
    """Rows the scan kernel streams per batch: every list once per group of ≤ `group` of its probing
    queries, Σ_l ⌈c_l / group⌉·|l| (≥ the distinct-list rows when a list is probed by > group queries)."""
    sizes = np.diff(index._offsets)
    c = np.bincount(probes[probes >= 0].ravel(), minlength=len(sizes))
    return int((-(-c // group) * sizes).sum())


def flat_ground_truth(torch, hipann, d: int, metric: int, xq, k: int, n_total: int, rank: int, world: int,
                      ivf_info_tensor=None):
    """Exact top-k over the whole (sharded) database with the Flat kernels; labels mapped through the
    IVF shard's ids.  Returns an (nq, k) numpy array on rank 0 (None elsewhere)."""
    import torch.distributed as dist

    cen, codes, ids = ivf_info_tensor._keep
    dev = codes.device
    nq = xq.shape[0]
    stream = torch.cuda.current_stream().cuda_stream
    flat = hipann.HipIndexFlatDevice(d, metric, codes.data_ptr(), codes.shape[0], dev.index, copy=False)
    D = torch.empty((nq, k), device=dev, dtype=torch.float32)
    I = torch.empty((nq, k), device=dev, dtype=torch.int64)
    flat.search_device(nq, xq.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)
    torch.cuda.synchronize()
    flat.close()
    lab = torch.where(I >= 0, ids[I.clamp_min(0)], I)
    if world > 1:
        Da = torch.empty((world, nq, k), device=dev, dtype=torch.float32)
        Ia = torch.empty((world, nq, k), device=dev, dtype=torch.int64)
        dist.all_gather_into_tensor(Da, D.contiguous())
        dist.all_gather_into_tensor(Ia, lab.contiguous())
        Do = torch.empty((nq, k), device=dev, dtype=torch.float32)
        Io = torch.empty((nq, k), device=dev, dtype=torch.int64)
        hipann.merge_topk_device(metric, world, nq, k, Da.data_ptr(), Ia.data_ptr(), Do.data_ptr(), Io.data_ptr(),
                                 stream)
        torch.cuda.synchronize()
        lab = Io
    return lab.cpu().numpy() if rank == 0 else None
