"""sharded — one-process-per-GPU sharded search with ONE all-gather of per-shard top-k.

The reference has no multi-device code (SURVEY §2a "Parallelism and communication"); this is the
MI355X-native addition of SURVEY §8e:

* Flat: database rows split into contiguous ranges, one per rank (``shard_bounds``);
* IVFFlat: whole inverted lists dealt to ranks by size-balanced greedy assignment, largest first onto
  the least-loaded rank (``assign_lists``) — every rank holds the 3 MB coarse quantizer, computes the probe lists
  of its slice of the batch, one all-gather of the probe lists (``PartitionedProbes``) gives every rank the whole
  batch's, and each rank scans only the probed lists it owns.

Every rank searches only its shard on its own GPU, with labels already global.  Its top-k is packed
into one buffer per rank — ``[labels int64 nq·k][distances fp32 nq·k]``, 12·nq·k bytes (123 KB at
nq = 1024, k = 10) — and moved by a single ``all_gather_into_tensor`` over RCCL (xGMI), then merged on
every rank with the same (distance, label) order the single-GPU path uses
(``hipann_merge_topk_packed_device``).  There is no other data-path collective: queries are
replicated, the database never moves.
"""
from __future__ import annotations

from typing import Callable, Sequence, Tuple

import numpy as np


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row range [lo, hi) of `rank` (labels of the shard are lo + local row)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    return rank * n // world, (rank + 1) * n // world


def assign_lists(list_sizes: Sequence[int], world: int) -> np.ndarray:
    """Size-balanced list → rank map: lists sorted by size (largest first, stable), each dealt to the
    currently least-loaded rank (ties → lowest rank).  The same rule hipann_ivf_create uses for the
    in-process multi-device index (ivf.cpp)."""
    sizes = np.asarray(list_sizes, np.int64)
    owner = np.zeros(len(sizes), np.int64)
    if world <= 1:
        return owner
    load = np.zeros(world, np.int64)
    for l in np.argsort(-sizes, kind="stable"):
        r = int(np.argmin(load))
        owner[l] = r
        load[r] += sizes[l]
    return owner


def part_bytes(nq: int, k: int) -> int:
    """Bytes of one rank's packed top-k: int64 labels then fp32 distances, padded to 8 B."""
    b = nq * k * 12
    return (b + 7) // 8 * 8


def unpack_parts(gathered, nq: int, k: int):
    """[world][part_bytes] uint8 → (D [world][nq][k] fp32, I [world][nq][k] int64) (host merges, tests)."""
    world = gathered.shape[0]
    import torch

    lab = gathered[:, : nq * k * 8].contiguous().view(torch.int64).reshape(world, nq, k)
    dis = gathered[:, nq * k * 8: nq * k * 12].contiguous().view(torch.float32).reshape(world, nq, k)
    return dis, lab


class ShardedSearch:
    """Glue between a per-rank search and the single all-gather + merge.

    ``local_search(xq, D, I)``: writes this rank's top-k into the (nq, k) views D (fp32) and I (int64,
    GLOBAL labels, −1 pads) — views into the packed buffer the collective sends.
    ``merge(gathered, nq, k) -> (D, I)``: merge of the [world][part_bytes] uint8 buffer (the GPU path
    passes ``merge_packed_device_torch``; CPU tests a host restatement via ``unpack_parts``).
    Works with any torch.distributed backend (nccl = RCCL on ROCm; gloo for CPU tests).
    ``gather_at_world1``: run the collective + merge even with one rank (the RCCL path's own test on a
    one-GPU box; a single rank otherwise returns its local top-k directly).
    """

    def __init__(self, local_search: Callable, merge: Callable, nq: int, k: int, device, group=None,
                 gather_at_world1: bool = False):
        import torch
        import torch.distributed as dist

        self.local_search = local_search
        self.merge = merge
        self.group = group
        self.nq, self.k = nq, k
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.pb = part_bytes(nq, k)
        self.packed = torch.zeros(self.pb, dtype=torch.uint8, device=device)
        self.I = self.packed[: nq * k * 8].view(torch.int64).view(nq, k)
        self.D = self.packed[nq * k * 8: nq * k * 12].view(torch.float32).view(nq, k)
        self.collective = self.world > 1 or (gather_at_world1 and dist.is_initialized())
        self.gathered = torch.empty((self.world, self.pb), dtype=torch.uint8, device=device) if self.collective \
            else None

    def search(self, xq):
        import torch.distributed as dist

        if not self.collective:  # one rank: the search writes fresh tensors (no packed buffer, no copy)
            import torch

            D = torch.empty((self.nq, self.k), dtype=torch.float32, device=self.packed.device)
            I = torch.empty((self.nq, self.k), dtype=torch.int64, device=self.packed.device)
            self.local_search(xq, D, I)
            return D, I
        self.local_search(xq, self.D, self.I)
        if self.packed.is_cuda and dist.get_backend(self.group) == "nccl":
            # RCCL: one collective straight into the buffer the merge reads
            dist.all_gather_into_tensor(self.gathered.view(-1), self.packed, group=self.group)
        else:  # gloo (CPU tests; GPU tests with several ranks on one device): the same bytes via host memory
            host = self.packed.cpu()
            parts = [torch_empty_like_cpu(host) for _ in range(self.world)]
            dist.all_gather(parts, host, group=self.group)
            for r, p in enumerate(parts):
                self.gathered[r].copy_(p)
        return self.merge(self.gathered, self.nq, self.k)


def query_bounds(nq: int, rank: int, world: int) -> Tuple[int, int]:
    """The slice of the batch whose coarse step `rank` computes (contiguous, as shard_bounds)."""
    return shard_bounds(nq, rank, world)


def coarse_partition_ok(nq: int, world: int) -> bool:
    """Partition the coarse step only when every rank's slice keeps FAISS's BLAS form (>= 20 queries,
    distance_compute_blas_threshold): a query's probe list then does not depend on the slice it was computed in."""
    return world > 1 and nq // world >= 20


class PartitionedProbes:
    """The IVF coarse step partitioned over ranks: rank r computes the probe lists of its slice of the
    batch (``coarse(q_slice, probes_out)``, e.g. hipann_ivf_coarse_device), and ONE all-gather of the padded
    [world][ceil(nq/world)][nprobe] int64 lists (256 KB at nq 1024, nprobe 32) gives every rank the whole batch's —
    instead of every rank running the same coarse quantizer over all nq queries.  The lists are bit-identical to the
    replicated step's while ``coarse_partition_ok``."""

    def __init__(self, coarse: Callable, nq: int, nprobe: int, device, group=None):
        import torch
        import torch.distributed as dist

        self.coarse = coarse
        self.group = group
        self.nq, self.nprobe = nq, nprobe
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.rows = -(-nq // self.world)
        self.lo, self.hi = query_bounds(nq, self.rank, self.world)
        self.local = torch.full((self.rows, nprobe), -1, dtype=torch.int64, device=device)
        self.gathered = torch.empty((self.world, self.rows, nprobe), dtype=torch.int64, device=device)
        self.bounds = [query_bounds(nq, r, self.world) for r in range(self.world)]
        self.out = torch.empty((nq, nprobe), dtype=torch.int64, device=device)

    def probes(self, xq):
        """(nq, nprobe) int64 probe lists of the whole batch xq on every rank."""
        import torch.distributed as dist

        m = self.hi - self.lo
        if m:
            self.coarse(xq[self.lo:self.hi], self.local[:m])
        if self.world == 1:
            return self.local[: self.nq]
        if self.local.is_cuda and dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self.gathered.view(-1), self.local.view(-1), group=self.group)
        else:  # gloo: through host memory
            host = self.local.cpu()
            parts = [torch_empty_like_cpu(host) for _ in range(self.world)]
            dist.all_gather(parts, host, group=self.group)
            for r, p in enumerate(parts):
                self.gathered[r].copy_(p)
        for r, (lo, hi) in enumerate(self.bounds):
            self.out[lo:hi].copy_(self.gathered[r, : hi - lo])
        return self.out


def torch_empty_like_cpu(t):
    import torch

    return torch.empty_like(t, device="cpu")


def collective_tensor(t, op, group=None):
    """Run an in-place collective (``op(tensor)``: broadcast / all_reduce) on `t`, through host memory when
    the backend is not RCCL (gloo cannot reduce device tensors in every build)."""
    import torch.distributed as dist

    if not t.is_cuda or dist.get_backend(group) == "nccl":
        op(t)
        return t
    h = t.cpu()
    op(h)
    t.copy_(h)
    return t


def merge_packed_device_torch(hipann, metric: int):
    """The GPU merge of packed parts as a ``merge`` callable for ShardedSearch."""
    import torch

    def merge(gathered, nq, k):
        world, pb = gathered.shape
        D = torch.empty((nq, k), device=gathered.device, dtype=torch.float32)
        I = torch.empty((nq, k), device=gathered.device, dtype=torch.int64)
        hipann.merge_topk_packed_device(metric, world, nq, k, gathered.data_ptr(), pb, D.data_ptr(), I.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream)
        return D, I

    return merge
