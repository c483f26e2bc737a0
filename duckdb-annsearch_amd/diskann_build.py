"""diskann_build — synthetic DiskANN inputs for the C4 benchmark, built on the GPU.

The extension builds its graph with the Rust `diskann` crate (Vamana, out of scope here)
and stores it in a `.diskann` v2 file (rust_lib/src/file_format.rs:3-74) with an optional SQ8
trailer (index_manager.rs:513-533).  The benchmark needs a navigable graph of the same shape —
N x R u32 adjacency padded with u32::MAX, one entry point — over 1M x 1536 rows without that
crate, so this module builds one on the device with torch (setup only; nothing here is timed):

  * R - n_random nearest neighbours per row (exact within two overlapping k-means cells: each row is
    assigned to its two nearest cells and gets the nearest rows of both), sorted by distance;
  * n_random uniformly random long-range edges (the role of Vamana's alpha-pruned far edges);
  * entry point = the medoid (row nearest to the mean), as DiskANN does.

sq8_encode restates the extension's codec (rust_lib/src/provider.rs:161-210) on the device:
per-dimension min/max, scale = max - min (1 when 0), code = clamp(round((v - min) / scale * 255))
with round-half-away-from-zero (Rust f32::round) — (v - min) / scale * 255 is non-negative, so
floor(x + 0.5) is that rounding.
"""
from __future__ import annotations


def sq8_encode(torch, x, chunk: int = 1 << 17):
    """x: (n, d) CUDA fp32 → (codes uint8 (n, d), mins fp32 (d,), scale fp32 (d,))."""
    mins = x.min(0).values
    maxs = x.max(0).values
    scale = maxs - mins
    scale = torch.where(scale == 0, torch.ones_like(scale), scale)
    codes = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    for r0 in range(0, x.shape[0], chunk):
        v = (x[r0:r0 + chunk] - mins) / scale * 255.0
        codes[r0:r0 + chunk] = torch.floor(v + 0.5).clamp_(0, 255).to(torch.uint8)
    return codes, mins.contiguous(), scale.contiguous()


def _sqnorm(x):
    return (x * x).sum(1)


def knn_graph(torch, x, R: int = 64, n_random: int = 16, ncells: int = 1024, iters: int = 4, seed: int = 8,
              chunk: int = 65536):
    """x: (n, d) CUDA fp32.  Returns (adjacency (n, R) int64 CUDA tensor of row ids, medoid id)."""
    n, d = x.shape
    dev = x.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    n_knn = R - n_random
    xn = _sqnorm(x)
    # k-means cells (a few Lloyd iterations from a random sample)
    ncells = max(1, min(ncells, n // 64))
    cen = x[torch.randperm(n, generator=g, device=dev)[:ncells]].clone()

    def nearest_cells(k):
        out = torch.empty((n, k), dtype=torch.int64, device=dev)
        cn = _sqnorm(cen)
        for r0 in range(0, n, chunk):
            dd = cn[None, :] - 2.0 * (x[r0:r0 + chunk] @ cen.T)
            out[r0:r0 + chunk] = torch.topk(dd, k, dim=1, largest=False).indices
        return out

    for _ in range(iters):
        a = nearest_cells(1)[:, 0]
        cnt = torch.bincount(a, minlength=ncells).to(torch.float32)
        s = torch.zeros_like(cen).index_add_(0, a, x)
        keep = cnt > 0
        cen[keep] = s[keep] / cnt[keep, None]
    two = nearest_cells(2)  # (n, 2): primary and secondary cell
    kk = n_knn + 1  # + self
    cand_i = torch.full((n, 2, kk), -1, dtype=torch.int64, device=dev)
    cand_d = torch.full((n, 2, kk), float("inf"), dtype=torch.float32, device=dev)
    flat_cell = two.reshape(-1)
    order = torch.argsort(flat_cell, stable=True)
    bounds = torch.searchsorted(flat_cell[order], torch.arange(ncells + 1, device=dev)).cpu().tolist()
    for c in range(ncells):
        sel = order[bounds[c]:bounds[c + 1]]
        if sel.numel() == 0:
            continue
        rows, slot = sel // 2, sel % 2
        xc = x[rows]
        nc = xn[rows]
        kc = min(kk, rows.numel())
        for s0 in range(0, rows.numel(), 8192):  # bounded (8192 x cell) distance tiles
            dd = nc[s0:s0 + 8192, None] + nc[None, :] - 2.0 * (xc[s0:s0 + 8192] @ xc.T)
            v, j = torch.topk(dd, kc, dim=1, largest=False)
            cand_i[rows[s0:s0 + 8192], slot[s0:s0 + 8192], :kc] = rows[j]
            cand_d[rows[s0:s0 + 8192], slot[s0:s0 + 8192], :kc] = v
    ci = cand_i.reshape(n, -1)
    cd = cand_d.reshape(n, -1)
    # drop self and duplicates (the same pair found in both cells), keep the n_knn nearest
    si, perm = torch.sort(ci, dim=1)
    sd = torch.gather(cd, 1, perm)
    dup = torch.zeros_like(si, dtype=torch.bool)
    dup[:, 1:] = si[:, 1:] == si[:, :-1]
    me = torch.arange(n, device=dev)[:, None]
    sd = torch.where(dup | (si == me) | (si < 0), torch.full_like(sd, float("inf")), sd)
    v, j = torch.topk(sd, n_knn, dim=1, largest=False)
    knn = torch.gather(si, 1, j)
    knn = torch.where(torch.isinf(v), torch.full_like(knn, -1), knn)
    rnd = torch.randint(0, n - 1, (n, n_random), generator=g, device=dev)
    rnd = rnd + (rnd >= me).to(torch.int64)  # skip self
    adj = torch.cat([knn, rnd], 1)
    # -1 holes (tiny cells) → move to the tail as u32::MAX padding
    hole = adj < 0
    key = hole.to(torch.int64) * 2 * R + torch.arange(R, device=dev)[None, :]
    adj = torch.gather(adj, 1, torch.argsort(key, dim=1))
    mean = x.mean(0, keepdim=True)
    medoid = int(torch.argmin(_sqnorm(x - mean)))
    return adj, medoid


def adjacency_u32(torch, adj):
    """(n, R) int64 with −1 holes → numpy uint32 with u32::MAX padding (file_format.rs:3-18)."""
    import numpy as np

    a = adj.cpu().numpy()
    out = a.astype(np.uint32)
    out[a < 0] = np.uint32(0xFFFFFFFF)
    return out


def exact_topk(torch, x, q, k: int, metric: int = 0, chunk: int = 1 << 18):
    """Exact top-k ids of q (nq, d) over x (n, d) in fp64-safe decomposed fp32 (ground truth for recall)."""
    nq = q.shape[0]
    best_d = torch.full((nq, k), float("inf"), device=x.device)
    best_i = torch.full((nq, k), -1, dtype=torch.int64, device=x.device)
    qn = _sqnorm(q)
    for r0 in range(0, x.shape[0], chunk):
        xc = x[r0:r0 + chunk]
        if metric == 0:
            dd = qn[:, None] + _sqnorm(xc)[None, :] - 2.0 * (q @ xc.T)
        else:
            dd = -(q @ xc.T)
        v, j = torch.topk(dd, min(k, xc.shape[0]), dim=1, largest=False)
        allv = torch.cat([best_d, v], 1)
        alli = torch.cat([best_i, j + r0], 1)
        best_d, p = torch.topk(allv, k, dim=1, largest=False)
        best_i = torch.gather(alli, 1, p)
    return best_i
