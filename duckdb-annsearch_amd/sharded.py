"""sharded — one-process-per-GPU sharded search with a single all-gather of per-shard top-k.

The reference has no multi-device code (SURVEY §2a "Parallelism and communication"); this is the
MI355X-native addition of SURVEY §8e: database rows (Flat) or the rows of every IVF list are split
into contiguous ranges, one per rank; every rank searches only its range on its own GPU; the per-rank
top-k (nq × k × (4 + 8) bytes — 123 KB at nq = 1024, k = 10) is all-gathered over RCCL (xGMI) and
merged on every rank with the same (distance, label) order the single-GPU path uses.  There is no
other data-path collective: the queries are replicated, the database never moves.
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous row range [lo, hi) of `rank` (labels of the shard are lo + local row)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    return rank * n // world, (rank + 1) * n // world


class ShardedSearch:
    """Glue between a per-rank search and the all-gather + merge.

    ``local_search(xq) -> (D, I)``: this rank's top-k, I holding GLOBAL labels (−1 pads).
    ``merge(D_all, I_all) -> (D, I)``: merge of [world][nq][k] partials (the GPU path passes
    hipann.merge_topk_device; tests may pass a host implementation of the same order).
    Works with any torch.distributed backend (nccl = RCCL on ROCm; gloo for CPU tests).
    """

    def __init__(self, local_search: Callable, merge: Callable, group=None):
        import torch.distributed as dist

        self.local_search = local_search
        self.merge = merge
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def search(self, xq):
        import torch
        import torch.distributed as dist

        D, I = self.local_search(xq)
        if self.world == 1:
            return D, I
        if D.is_cuda:  # RCCL: gather straight into the [world][nq][k] buffers the merge reads
            if getattr(self, "_bufs", None) is None or self._bufs[0].shape[1:] != D.shape:
                self._bufs = (torch.empty((self.world, *D.shape), device=D.device, dtype=D.dtype),
                              torch.empty((self.world, *I.shape), device=I.device, dtype=I.dtype))
            Da, Ia = self._bufs
            dist.all_gather_into_tensor(Da, D.contiguous(), group=self.group)
            dist.all_gather_into_tensor(Ia, I.contiguous(), group=self.group)
            return self.merge(Da, Ia)
        Dl = [torch.empty_like(D) for _ in range(self.world)]
        Il = [torch.empty_like(I) for _ in range(self.world)]
        dist.all_gather(Dl, D.contiguous(), group=self.group)
        dist.all_gather(Il, I.contiguous(), group=self.group)
        return self.merge(torch.stack(Dl), torch.stack(Il))


def merge_topk_device_torch(hipann, metric: int):
    """The GPU merge as a ``merge`` callable for ShardedSearch (torch CUDA tensors in / out)."""
    import torch

    def merge(D_all, I_all):
        world, nq, k = D_all.shape
        D = torch.empty((nq, k), device=D_all.device, dtype=torch.float32)
        I = torch.empty((nq, k), device=D_all.device, dtype=torch.int64)
        hipann.merge_topk_device(metric, world, nq, k, D_all.data_ptr(), I_all.data_ptr(), D.data_ptr(),
                                 I.data_ptr(), torch.cuda.current_stream().cuda_stream)
        return D, I

    return merge
