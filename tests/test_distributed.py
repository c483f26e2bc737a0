"""World-size-2 gloo test of the sharded (multi-GPU) search orchestration on the CPU.

Each rank searches its contiguous row range (the oracle stands in for the per-GPU shard search: it is
the same semantic contract the GPU parity tests check), the per-rank top-k is all-gathered through
ShardedSearch (the class bench.py uses over RCCL), and merged with a host restatement of
merge_parts_topk's (distance, label) order.  The result must equal the single-process search over the
whole database.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def host_merge(D_all, I_all, metric):
    """Host restatement of merge_parts_topk: k best of the union by (key, label), key = D (L2) or −D (IP)."""
    import torch

    world, nq, k = D_all.shape
    D = np.asarray(D_all.permute(1, 0, 2).reshape(nq, world * k))
    I = np.asarray(I_all.permute(1, 0, 2).reshape(nq, world * k))
    key = D if metric == 0 else -D
    outD = np.full((nq, k), np.inf if metric == 0 else -np.inf, np.float32)
    outI = np.full((nq, k), -1, np.int64)
    for q in range(nq):
        cand = [(key[q, j], I[q, j]) for j in range(world * k) if I[q, j] >= 0]
        cand.sort()
        for j, (kv, lab) in enumerate(cand[:k]):
            outD[q, j] = kv if metric == 0 else -kv
            outI[q, j] = lab
    return torch.from_numpy(outD), torch.from_numpy(outI)


def _worker(rank, world, port, metric, result_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from sharded import ShardedSearch, shard_bounds
    from _data import faiss_metal_case

    dist.init_process_group("gloo", rank=rank, world_size=world)
    xb, xq = faiss_metal_case(3001, 25, 48)
    lo, hi = shard_bounds(len(xb), rank, world)

    def local(q):
        D, I = O.flat_search(xb[lo:hi], q.numpy(), 12, metric, label_offset=lo)
        I = np.where(I >= 0, I, -1)
        return torch.from_numpy(D), torch.from_numpy(I)

    s = ShardedSearch(local, lambda Da, Ia: host_merge(Da, Ia, metric))
    D, I = s.search(torch.from_numpy(xq))
    if rank == 0:
        np.savez(result_path, D=D.numpy(), I=I.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("metric", [0, 1])
def test_sharded_search_gloo_world2(tmp_path, metric):
    import torch.multiprocessing as mp
    from oracle import oracle as O
    from _data import faiss_metal_case

    out = tmp_path / "res.npz"
    mp.spawn(_worker, args=(2, _free_port(), metric, str(out)), nprocs=2, join=True)
    r = np.load(out)
    xb, xq = faiss_metal_case(3001, 25, 48)
    Do, Io = O.flat_search(xb, xq, 12, metric)
    assert np.array_equal(r["I"], Io)
    assert np.allclose(r["D"], Do, rtol=1e-6)


def test_shard_bounds_cover_rows():
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    from sharded import shard_bounds
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
