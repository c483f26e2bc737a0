"""ivf_build — build an IVFFlat shard on the GPU for the benchmark / integration tests.

The extension builds its IVF index on the CPU with FAISS (faiss_index.cpp:302-332: train on a
stride sample, then add) and copies it to the GPU (index_cpu_to_metal_ivf,
MetalIndexIVFFlat.mm:283-326).  FAISS is absent here, so this module does the same work on the GPU
(SURVEY §8f rank 4): k-means over a 256·nlist-point sample (FAISS's default max_points_per_centroid,
25 iterations, k-means++ init) through the C ABI (hipann_ivf_train_device: the same entry point the extension's
CREATE INDEX would call, faiss_index.cpp:302-319), assignment of every row with the Flat kernels (k = 1),
a stable counting sort into list-contiguous storage, and hipann_ivf_create_device on the result.
``kmeans_torch`` is the r01-r03 torch implementation, kept as the comparison the C-ABI training is held to.

Training sample: the first 256·nlist rows of the database (identical for every world size, so the
1/2/4/8-GPU runs search the same lists).

Multi-GPU: rank 0 trains and broadcasts the centroids, then
  * ``build_ivf_list_shard`` (the default): whole lists are dealt to ranks by size
    (sharded.assign_lists — the list sizes come from each rank counting its row range, summed by one
    all-reduce at build time); every rank regenerates the database chunk by chunk (the generators are
    chunk-seeded, so no rows travel between GPUs), assigns it, and keeps the rows of the lists it owns;
  * ``build_ivf_shard`` with world > 1: every rank assigns and stores only its own row range, so list l
    is split across ranks by row range (kept for comparison: perfectly balanced bytes, shorter lists).
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
    """IVF training through the C ABI (hipann_ivf_train_device): k-means++ init + Lloyd on the GPU, no torch in the
    loop.  x: (m, d) CUDA fp32 (m <= 256·nlist: the whole of it is the training set)."""
    m, d = x.shape
    cen = torch.empty((nlist, d), device=x.device, dtype=torch.float32)
    torch.cuda.synchronize()
    hipann.ivf_train_device(d, nlist, m, x.data_ptr(), cen.data_ptr(), metric=metric, train_sample=0, niter=niter,
                            seed=seed, init=hipann.KMEANS_INIT_PLUSPLUS if init == "kmeans++" else hipann.KMEANS_INIT_RANDOM,
                            device=x.device.index, stream=torch.cuda.current_stream().cuda_stream)
    return cen


def kmeans_torch(torch, hipann, x, nlist: int, niter: int = 25, seed: int = 1234, metric: int = 0,
                 init: str = "kmeans++"):
    """The r01-r03 Lloyd k-means in torch (assignment through the Flat kernels).  x: (m, d) CUDA fp32."""
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
                    world: int, centres_seed: int = 1234, train_points_per_list: int = 256, train=None):
    """Returns (HipIndexIVFFlat over this rank's rows, info dict)."""
    import torch.distributed as dist

    dev = xb.device
    n_local, d = xb.shape
    # ---- train (rank 0, on the first 256·nlist rows; rank 0 holds them in both layouts) ----
    if rank == 0:
        m = min(n_local, train_points_per_list * nlist)
        cen = (train or kmeans)(torch, hipann, xb[:m].contiguous(), nlist, seed=centres_seed)
    else:
        cen = torch.empty((nlist, d), device=dev, dtype=torch.float32)
    if world > 1:
        dist.broadcast(cen, 0)
    cen = cen.contiguous()
    assign = assign_rows(torch, hipann, cen, xb, metric)
    # ---- list-contiguous storage (stable counting sort) ----
    order = torch.sort(assign, stable=True).indices
    counts = torch.bincount(assign, minlength=nlist)
    codes = torch.empty_like(xb)
    for s in range(0, n_local, ASSIGN_CHUNK):
        e = min(n_local, s + ASSIGN_CHUNK)
        codes[s:e] = xb[order[s:e]]
    ids = (order + row0).contiguous()
    del order, assign
    info = {"shard": "rows" if world > 1 else "single"}
    return _make_index(torch, hipann, d, metric, nlist, nprobe, cen, counts, codes, ids, dev, info)


ASSIGN_CHUNK = 1_000_000


def assign_rows(torch, hipann, cen, x, metric: int):
    """Nearest centroid of every row of x (Flat kernels, k = 1, chunks of 1M rows) → int64 CUDA tensor."""
    n, d = x.shape
    dev = x.device
    stream = torch.cuda.current_stream().cuda_stream
    assign = torch.empty((n,), device=dev, dtype=torch.int64)
    qidx = hipann.HipIndexFlatDevice(d, metric, cen.data_ptr(), cen.shape[0], dev.index, copy=False)
    m = min(n, ASSIGN_CHUNK)
    Dc = torch.empty((m, 1), device=dev, dtype=torch.float32)
    Ic = torch.empty((m, 1), device=dev, dtype=torch.int64)
    for s in range(0, n, ASSIGN_CHUNK):
        e = min(n, s + ASSIGN_CHUNK)
        qidx.search_device(e - s, x[s:e].data_ptr(), 1, Dc.data_ptr(), Ic.data_ptr(), stream)
        assign[s:e].copy_(Ic[:e - s, 0])
    torch.cuda.synchronize()
    qidx.close()
    return assign


def _make_index(torch, hipann, d, metric, nlist, nprobe, cen, counts, codes, ids, dev, info):
    offsets = np.zeros(nlist + 1, np.int64)
    offsets[1:] = np.cumsum(counts.cpu().numpy())
    index = hipann.HipIndexIVFFlat.from_device(d, metric, nlist, nprobe, cen.data_ptr(), offsets, ids.data_ptr(),
                                               codes.data_ptr(), dev.index, copy=False)
    index._keep = (cen, codes, ids)  # borrowed by the library
    index._offsets = offsets
    sizes = np.diff(offsets)
    info.update({"nlist": nlist, "nprobe": nprobe, "list_size_min": int(sizes.min()),
                 "list_size_max": int(sizes.max()), "list_size_mean": float(sizes.mean()),
                 "rows_local": int(offsets[-1])})
    return index, info


def build_ivf_list_shard(torch, hipann, gen_rows, n_total: int, d: int, nlist: int, nprobe: int, metric: int,
                         rank: int, world: int, dev, centres_seed: int = 1234, train_points_per_list: int = 256):
    """List-sharded IVF shard of rank `rank`.  ``gen_rows(out, row0)`` fills `out` with
    global rows [row0, row0 + len(out)) (deterministic, chunk-seeded).  Returns (index over the owned
    lists, info)."""
    import torch.distributed as dist

    from sharded import assign_lists, collective_tensor, shard_bounds

    m = min(n_total, train_points_per_list * nlist)
    if rank == 0:
        sample = gen_rows(torch.empty((m, d), device=dev, dtype=torch.float32), 0)
        cen = kmeans(torch, hipann, sample, nlist, seed=centres_seed)
        del sample
    else:
        cen = torch.empty((nlist, d), device=dev, dtype=torch.float32)
    if world > 1:
        collective_tensor(cen, lambda t: dist.broadcast(t, 0))
    cen = cen.contiguous()
    buf = torch.empty((min(ASSIGN_CHUNK, n_total), d), device=dev, dtype=torch.float32)
    # list sizes: each rank counts its own row range, one all-reduce sums them (build time only)
    lo, hi = shard_bounds(n_total, rank, world)
    counts = torch.zeros(nlist, device=dev, dtype=torch.int64)
    for s in range(lo, hi, ASSIGN_CHUNK):
        e = min(hi, s + ASSIGN_CHUNK)
        x = gen_rows(buf[:e - s], s)
        counts += torch.bincount(assign_rows(torch, hipann, cen, x, metric), minlength=nlist)
    if world > 1:
        collective_tensor(counts, dist.all_reduce)
    owner = assign_lists(counts.cpu().numpy(), world)
    mine = torch.from_numpy(owner == rank).to(dev)
    keep_x, keep_i, keep_a = [], [], []
    for s in range(0, n_total, ASSIGN_CHUNK):
        e = min(n_total, s + ASSIGN_CHUNK)
        x = gen_rows(buf[:e - s], s)
        a = assign_rows(torch, hipann, cen, x, metric)
        sel = torch.nonzero(mine[a]).squeeze(1)
        keep_x.append(x[sel])
        keep_i.append(sel + s)
        keep_a.append(a[sel])
    del buf
    a = torch.cat(keep_a)
    order = torch.sort(a, stable=True).indices  # rows of a list stay in ascending global id (insertion order)
    codes = torch.cat(keep_x)[order].contiguous()
    ids = torch.cat(keep_i)[order].contiguous()
    del keep_x, keep_i, keep_a
    local_counts = torch.bincount(a, minlength=nlist)
    info = {"shard": "lists", "lists_owned": int(mine.sum())}
    return _make_index(torch, hipann, d, metric, nlist, nprobe, cen, local_counts, codes, ids, dev, info)


def scan_bytes(index, probes: np.ndarray, d: int, row_bytes: float = None) -> float:
    """Algorithmic HBM bytes of one batch's list scan on this shard: every distinct probed list read
    once, |l|·row_bytes — by default SURVEY §8d's |l|·(4d + 8) (fp32 codes + label)."""
    sizes = np.diff(index._offsets)
    distinct = np.unique(probes[probes >= 0])
    return float(sizes[distinct].sum()) * (4 * d + 8 if row_bytes is None else row_bytes)


def scan_pairs(index, probes: np.ndarray) -> int:
    """(query, row) distance evaluations of one batch on this shard: Σ_q Σ_p |l(q, p)|."""
    sizes = np.diff(index._offsets)
    p = probes[probes >= 0]
    return int(sizes[p].sum())


def half_scan_groups(d: int, mode: int = 2, gemm: bool = False) -> tuple:
    """(narrow, wide, gemm) query-group sizes of the fp16 form's scan (ivf_mfma.hip mh_group / mh_group_wide /
    mh_group_packed: the queries' LDS image, two fp16 terms or the high term only, in 160 KiB; GEMM items of 256) for
    HIPANN_IVF_WIDE = mode (2 default: every list at least wide, narrow 0; 1: wide above the narrow size; 0: no wide
    items) and HIPANN_IVF_GEMM (gemm)."""
    nsup = -(-(-(-d // 32)) // 6) * 6
    g = min(48, (163840 // ((2 * nsup * 16 + 8) * 4)) // 16 * 16)
    w = min(96, (163840 // ((nsup * 16 + 8) * 4 + 8)) // 16 * 16)
    if not mode or w <= g or g < 16:
        return g, 0, 0
    return (0 if mode == 2 else g), w, (256 if gemm and w >= 16 else 0)


def i8_scan_groups(d: int) -> tuple:
    """(narrow, wide, gemm) query-group sizes of the int8 form's scan (ivf_mfma.hip ivf_mfma_i8_group: every item
    one-term, the queries' int8 units in 64-dim super-steps + (‖q‖², s_q) in 160 KiB, at most 96)."""
    nsup = -(-(-(-d // 64)) // 6) * 6
    return 0, min(96, (163840 // ((nsup * 16 + 8) * 4 + 8)) // 16 * 16), 0


def scan_group_rows(index, probes: np.ndarray, group: int = 32, wide: int = 0, gemm: int = 0) -> int:
    """Rows the scan kernel streams per batch: every list once per group of its probing queries,
    Σ_l ⌈c_l / g_l⌉·|l| with g_l = `gemm` for a list probed by more than the wide size (when gemm > 0), `wide` for
    one probed by more than `group` (when wide > 0), else `group` (≥ the distinct-list rows when a list is probed by
    more queries than one group holds) — ivf_ngroups (common.hpp)."""
    sizes = np.diff(index._offsets)
    c = np.bincount(probes[probes >= 0].ravel(), minlength=len(sizes))
    g = np.full_like(c, group)
    if wide > 0:
        g = np.where(c > group, wide, g)
    if gemm > 0:
        g = np.where(c > (wide if wide > 0 else group), gemm, g)
    g = np.maximum(g, 1)
    return int((-(-c // g) * sizes).sum())


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
