"""World-size-2 tests of the sharded (multi-GPU) search orchestration.

CPU (gloo): each rank searches its shard — contiguous rows (Flat) or the whole lists it owns by the
size-balanced assignment (IVF) — with the oracle standing in for the per-GPU search (the same semantic
contract the GPU parity tests check); the per-rank top-k travels as ONE packed buffer through
ShardedSearch (the class bench.py uses over RCCL) and is merged with a host restatement of
merge_parts_topk's (distance, label) order.  The result must equal the single-process search.

GPU (gloo transport, both ranks on device 0 — RCCL needs one device per rank and the box has one):
the real per-rank HIP searches (HipIndexFlatDevice with label_offset; build_ivf_list_shard's
list-sharded IVF) and the device merge (hipann_merge_topk_packed_device), against the oracle over
the whole database.
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


def host_merge(gathered, nq, k, metric):
    """Host restatement of merge_parts_topk over the packed parts: k best of the union by (key, label),
    key = D (L2) or −D (IP)."""
    import torch
    from sharded import unpack_parts

    D_all, I_all = unpack_parts(gathered.cpu(), nq, k)
    world = D_all.shape[0]
    D = np.asarray(D_all.permute(1, 0, 2).reshape(nq, world * k))
    I = np.asarray(I_all.permute(1, 0, 2).reshape(nq, world * k))
    key = D if metric == 0 else -D
    outD = np.full((nq, k), np.inf if metric == 0 else -np.inf, np.float32)
    outI = np.full((nq, k), -1, np.int64)
    for q in range(nq):
        cand = sorted((key[q, j], I[q, j]) for j in range(world * k) if I[q, j] >= 0)
        for j, (kv, lab) in enumerate(cand[:k]):
            outD[q, j] = kv if metric == 0 else -kv
            outI[q, j] = lab
    return torch.from_numpy(outD), torch.from_numpy(outI)


def _setup(rank, world, port):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _worker_flat(rank, world, port, metric, result_path):
    dist = _setup(rank, world, port)
    import torch
    from oracle import oracle as O
    from sharded import ShardedSearch, shard_bounds
    from _data import faiss_metal_case

    xb, xq = faiss_metal_case(3001, 25, 48)
    lo, hi = shard_bounds(len(xb), rank, world)

    def local(q, D, I):
        Dl, Il = O.flat_search(xb[lo:hi], q.numpy(), 12, metric, label_offset=lo)
        D.copy_(torch.from_numpy(Dl))
        I.copy_(torch.from_numpy(np.where(Il >= 0, Il, -1)))

    s = ShardedSearch(local, lambda g, nq, k: host_merge(g, nq, k, metric), 25, 12, "cpu")
    D, I = s.search(torch.from_numpy(xq))
    if rank == 0:
        np.savez(result_path, D=D.numpy(), I=I.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("metric", [0, 1])
def test_sharded_flat_gloo_world2(tmp_path, metric):
    import torch.multiprocessing as mp
    from oracle import oracle as O
    from _data import faiss_metal_case

    out = tmp_path / "res.npz"
    mp.spawn(_worker_flat, args=(2, _free_port(), metric, str(out)), nprocs=2, join=True)
    r = np.load(out)
    xb, xq = faiss_metal_case(3001, 25, 48)
    Do, Io = O.flat_search(xb, xq, 12, metric)
    assert np.array_equal(r["I"], Io)
    assert np.allclose(r["D"], Do, rtol=1e-6)


def _worker_ivf_lists(rank, world, port, result_path):
    dist = _setup(rank, world, port)
    import torch
    from oracle import oracle as O
    from sharded import ShardedSearch, assign_lists
    from _data import build_ivf_lists, faiss_metal_case

    xb, xq = faiss_metal_case(6000, 30, 40)
    cen = np.ascontiguousarray(xb[::200][:30])
    off, ids, codes = build_ivf_lists(xb, cen)
    owner = assign_lists(np.diff(off), world)
    # this rank's lists only (the others empty), every centroid kept: the coarse step is replicated
    keep = np.concatenate([np.arange(off[l], off[l + 1]) for l in range(len(cen)) if owner[l] == rank])
    loff = np.zeros(len(cen) + 1, np.int64)
    loff[1:] = np.cumsum(np.where(owner == rank, np.diff(off), 0))

    def local(q, D, I):
        Dl, Il, _ = O.ivf_search(cen, loff, ids[keep], codes[keep], q.numpy(), 10, 7)
        D.copy_(torch.from_numpy(Dl))
        I.copy_(torch.from_numpy(np.where(Il >= 0, Il, -1)))

    s = ShardedSearch(local, lambda g, nq, k: host_merge(g, nq, k, 0), 30, 10, "cpu")
    D, I = s.search(torch.from_numpy(xq))
    if rank == 0:
        np.savez(result_path, D=D.numpy(), I=I.numpy(), owner=owner)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_ivf_list_ownership_gloo_world2(tmp_path):
    """IVF list sharding (north_star: "IVF lists shard across the GPUs"): every rank owns whole lists by
    size, scans the probed lists it owns; the merged result equals the single-index IVF search."""
    import torch.multiprocessing as mp
    from oracle import oracle as O
    from _data import build_ivf_lists, faiss_metal_case

    out = tmp_path / "res.npz"
    mp.spawn(_worker_ivf_lists, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    r = np.load(out)
    xb, xq = faiss_metal_case(6000, 30, 40)
    cen = np.ascontiguousarray(xb[::200][:30])
    off, ids, codes = build_ivf_lists(xb, cen)
    Do, Io, _ = O.ivf_search(cen, off, ids, codes, xq, 10, 7)
    assert np.array_equal(r["I"], Io)
    assert np.allclose(r["D"], Do, rtol=1e-6)
    assert set(np.unique(r["owner"]).tolist()) == {0, 1}


def test_assign_lists_balances_sizes():
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    from sharded import assign_lists
    rng = np.random.default_rng(3)
    sizes = rng.integers(7000, 12000, 1024)
    for w in (1, 2, 4, 8):
        owner = assign_lists(sizes, w)
        load = np.bincount(owner, weights=sizes, minlength=w)
        assert owner.min() == 0 and owner.max() == w - 1 if w > 1 else owner.max() == 0
        assert load.max() / load.mean() < 1.002


def test_packed_parts_layout():
    """One rank's packed top-k: int64 labels then fp32 distances, 8-B aligned; unpack restores both."""
    import torch
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    from sharded import part_bytes, unpack_parts
    for nq, k in ((1, 1), (3, 5), (1024, 10)):
        pb = part_bytes(nq, k)
        assert pb % 8 == 0 and pb >= 12 * nq * k
        g = torch.zeros((2, pb), dtype=torch.uint8)
        for r in range(2):
            g[r, : nq * k * 8].view(torch.int64).copy_(torch.arange(nq * k) + 100 * r)
            g[r, nq * k * 8: nq * k * 12].view(torch.float32).copy_(torch.arange(nq * k, dtype=torch.float32) / 2 + r)
        D, I = unpack_parts(g, nq, k)
        assert D.shape == (2, nq, k) and I.shape == (2, nq, k)
        assert int(I[1, 0, 0]) == 100 and float(D[1, 0, 0]) == 1.0


def test_shard_bounds_cover_rows():
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    from sharded import shard_bounds
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))


# ------------------------------------------------------------------------------------------------
# GPU: the real per-rank HIP searches + device merge, two ranks on device 0 (gloo transport)
# ------------------------------------------------------------------------------------------------
def _worker_gpu(rank, world, port, workload, result_path):
    dist = _setup(rank, world, port)
    import torch
    import hipann
    import bench
    from sharded import ShardedSearch, merge_packed_device_torch, shard_bounds

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, d, nq, k, metric = GPU_SHAPES[workload]
    stream = torch.cuda.current_stream().cuda_stream
    xq = bench.uniform_queries(torch, nq, d, dev)
    if workload.startswith("flat"):
        lo, hi = shard_bounds(n, rank, world)
        xb = torch.empty((hi - lo, d), device=dev)
        bench.gen_uniform_rows(torch, xb, lo, 42)
        index = hipann.HipIndexFlatDevice(d, metric, xb.data_ptr(), hi - lo, 0, copy=False, label_offset=lo)
        extra = {}
    else:
        from ivf_build import build_ivf_list_shard
        gen = lambda out, row0: bench.gen_uniform_rows(torch, out, row0, 42)  # noqa: E731
        index, info = build_ivf_list_shard(torch, hipann, gen, n, d, 64, 8, 0, rank, world, dev)
        cen, codes, ids = index._keep
        extra = {f"cen{rank}": cen.cpu().numpy(), f"ids{rank}": ids.cpu().numpy(), f"off{rank}": index._offsets,
                 f"codes{rank}": codes.cpu().numpy()}

    def local(q, D, I):
        index.search_device(nq, q.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)

    s = ShardedSearch(local, merge_packed_device_torch(hipann, metric), nq, k, dev)
    D, I = s.search(xq)
    torch.cuda.synchronize()
    np.savez(f"{result_path}.{rank}.npz", D=D.cpu().numpy(), I=I.cpu().numpy(), xq=xq.cpu().numpy(), **extra)
    dist.barrier()
    index.close()
    dist.destroy_process_group()


# (rows, d, nq, k, metric); flat_ip_c5: C5's per-GPU path (Flat IP, d = 768, the 1024-query batch) on
# 2 × 200k rows — the 100M × 768 / 8-GPU configuration's shard search, label offsets, all-gather and merge
GPU_SHAPES = {"flat": (60_000, 96, 200, 10, 0), "ivf_lists": (60_000, 96, 200, 10, 0),
              "flat_ip_c5": (400_000, 768, 1024, 10, 1)}


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["flat", "ivf_lists", "flat_ip_c5"])
def test_sharded_hip_world2_on_one_device(gpu, oracle, tmp_path, workload):
    """two processes, each running the real HIP shard search (Flat row shards with
    label_offset / list-sharded IVF from build_ivf_list_shard), one packed all-gather, the device merge
    kernel; the merged top-k equals the oracle's over the whole database (IVF: the lists the two ranks
    own partition the single index's lists, and the probe lists are the replicated coarse step's).
    flat_ip_c5 is C5's path (BASELINE configs[4]) at 400k rows: Flat IP, d 768, nq 1024, checked against
    the oracle on 128 of the queries."""
    import torch
    import torch.multiprocessing as mp
    import bench
    from _data import check_topk_parity

    res = str(tmp_path / "res")
    mp.spawn(_worker_gpu, args=(2, _free_port(), workload, res), nprocs=2, join=True)
    r0, r1 = np.load(res + ".0.npz"), np.load(res + ".1.npz")
    assert np.array_equal(r0["I"], r1["I"]) and np.array_equal(r0["D"], r1["D"])  # every rank merges the same
    n, d, nq, k, metric = GPU_SHAPES[workload]
    xb = bench.gen_uniform_rows(torch, torch.empty((n, d), device="cuda"), 0, 42).cpu().numpy()
    xq = r0["xq"]
    if workload == "flat_ip_c5":
        sub = slice(0, 128)
        Do, Io = oracle.flat_search(xb, xq[sub], k, metric)
        check_topk_parity(xb, xq[sub], r0["D"][sub], r0["I"][sub], Do, Io, metric)
        assert np.all(np.diff(r0["D"], axis=1) <= 0)  # IP: descending on every query
        return
    if workload == "flat":
        Do, Io = oracle.flat_search(xb, xq, 10)
    else:
        cen = r0["cen0"]
        assert np.array_equal(cen, r1["cen1"])
        len0, len1 = np.diff(r0["off0"]), np.diff(r1["off1"])
        assert not np.any((len0 > 0) & (len1 > 0))            # every list lives on one rank
        assert len0.sum() + len1.sum() == n and min(len0.sum(), len1.sum()) > 0.4 * n
        # the single index those two shards partition: list l from its owner, rows in ascending id
        parts = [(r0["off0"], r0["ids0"], r0["codes0"]), (r1["off1"], r1["ids1"], r1["codes1"])]
        off = np.zeros(len(cen) + 1, np.int64)
        off[1:] = np.cumsum(len0 + len1)
        ids = np.concatenate([p[1][p[0][l]:p[0][l + 1]] for l in range(len(cen)) for p in parts])
        codes = np.concatenate([p[2][p[0][l]:p[0][l + 1]] for l in range(len(cen)) for p in parts])
        assert np.array_equal(np.sort(ids), np.arange(n)) and np.array_equal(codes, xb[ids])
        assert all(np.all(np.diff(ids[off[l]:off[l + 1]]) > 0) for l in range(len(cen)))
        # the GPU assignment is the nearest centroid (up to fp32 near-ties) — the oracle's, mostly
        _, a = oracle.flat_search(cen, xb[ids], 1)
        lab = np.repeat(np.arange(len(cen)), np.diff(off))
        assert (a[:, 0] == lab).mean() > 0.999
        Do, Io, _ = oracle.ivf_search(cen, off, ids, codes, xq, 10, 8)
    check_topk_parity(xb, xq, r0["D"], r0["I"], Do, Io, 0)


# ------------------------------------------------------------------------------------------------
# RCCL: the all_gather_into_tensor branch of ShardedSearch (one rank: the box has one GPU)
# ------------------------------------------------------------------------------------------------
def _worker_rccl(rank, world, port, result_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import hipann
    import bench
    from sharded import ShardedSearch, merge_packed_device_torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    assert dist.get_backend() == "nccl"
    n, d, nq, k = 50_000, 128, 64, 10
    xb = torch.empty((n, d), device=dev)
    bench.gen_uniform_rows(torch, xb, 0, 42)
    xq = bench.uniform_queries(torch, nq, d, dev)
    index = hipann.HipIndexFlatDevice(d, 0, xb.data_ptr(), n, 0, copy=False)
    stream = torch.cuda.current_stream().cuda_stream

    def local(q, D, I):
        index.search_device(nq, q.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)

    s = ShardedSearch(local, merge_packed_device_torch(hipann, 0), nq, k, dev, gather_at_world1=True)
    assert s.collective and s.gathered.shape[0] == world
    D, I = s.search(xq)
    # the same search without the collective
    Dl = torch.empty((nq, k), device=dev)
    Il = torch.empty((nq, k), device=dev, dtype=torch.int64)
    local(xq, Dl, Il)
    torch.cuda.synchronize()
    np.savez(result_path, D=D.cpu().numpy(), I=I.cpu().numpy(), Dl=Dl.cpu().numpy(), Il=Il.cpu().numpy(),
             gathered=s.gathered.cpu().numpy(), packed=s.packed.cpu().numpy())
    index.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_rccl_all_gather_world1(gpu, tmp_path):
    """the RCCL branch of ShardedSearch.search (all_gather_into_tensor over the nccl backend,
    sharded.py) executes on the box — one rank on its one GPU, the packed top-k gathered by RCCL and merged by
    hipann_merge_topk_packed_device; the result equals the rank's own search, byte for byte."""
    import torch.multiprocessing as mp

    out = tmp_path / "rccl.npz"
    mp.spawn(_worker_rccl, args=(1, _free_port(), str(out)), nprocs=1, join=True)
    r = np.load(out)
    assert np.array_equal(r["gathered"][0], r["packed"])  # RCCL moved the packed buffer unchanged
    assert np.array_equal(r["I"], r["Il"]) and np.array_equal(r["D"], r["Dl"])


def test_bench_spawner_gloo_world2():
    """`bench.py --gpus 2` without a launcher starts the two ranks itself (torch.distributed.run
    child, no re-exec) — here the CPU self-test workload over gloo: both ranks rendezvous, all-gather their ranks
    and run the barrier / max-over-ranks timing; rank 0 prints one JSON line."""
    import json
    import subprocess

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", "selftest", "--steps",
                        "5", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["world_check"]["ranks_seen"] == [0, 1]
    assert js["world_check"]["backend"] == "gloo" and js["steps"] == 5


def test_bench_selftest_world1():
    """--gpus 1 stays one process (no spawner): the self-test line at N = 1."""
    import json
    import subprocess

    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--workload", "selftest", "--steps",
                        "3", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    js = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert js["n_gpus"] == 1 and js["world_check"]["ranks_seen"] == [0]


# ------------------------------------------------------------------------------------------------
# the IVF coarse step partitioned over ranks: PartitionedProbes
# ------------------------------------------------------------------------------------------------
def _worker_partitioned_probes(rank, world, port, result_path):
    dist = _setup(rank, world, port)
    import torch
    from oracle import oracle as O
    from sharded import PartitionedProbes
    from _data import faiss_metal_case

    xb, xq = faiss_metal_case(3000, 50, 40)
    cen = np.ascontiguousarray(xb[::100][:30])

    def coarse(q, out):  # FAISS quantizer->search(nq, x, nprobe) on this rank's slice
        _, P = O.flat_search(cen, q.numpy(), 7)
        out.copy_(torch.from_numpy(P))

    pp = PartitionedProbes(coarse, 50, 7, "cpu")
    P = pp.probes(torch.from_numpy(xq)).numpy().copy()
    if rank == 0:
        np.savez(result_path, P=P, rows=pp.rows)
    dist.barrier()
    dist.destroy_process_group()


def test_partitioned_probes_gloo_world2(tmp_path):
    """Each of two ranks computes the probe lists of its 25-query slice (>= 20: FAISS's BLAS form, as for the whole
    batch); one all-gather gives every rank the lists of all 50 queries, identical to the replicated coarse step."""
    import torch.multiprocessing as mp
    from oracle import oracle as O
    from _data import build_ivf_lists, faiss_metal_case

    out = tmp_path / "res.npz"
    mp.spawn(_worker_partitioned_probes, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    r = np.load(out)
    xb, xq = faiss_metal_case(3000, 50, 40)
    cen = np.ascontiguousarray(xb[::100][:30])
    off, ids, codes = build_ivf_lists(xb, cen)
    _, _, Po = O.ivf_search(cen, off, ids, codes, xq, 10, 7)
    assert np.array_equal(r["P"], Po) and int(r["rows"]) == 25


def test_coarse_partition_rule():
    sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
    from sharded import coarse_partition_ok, query_bounds
    assert coarse_partition_ok(1024, 8) and coarse_partition_ok(40, 2)
    assert not coarse_partition_ok(1024, 1) and not coarse_partition_ok(39, 2) and not coarse_partition_ok(100, 8)
    b = [query_bounds(1024, r, 8) for r in range(8)]
    assert b[0] == (0, 128) and b[-1] == (896, 1024)


def _worker_gpu_partitioned(rank, world, port, result_path):
    dist = _setup(rank, world, port)
    import torch
    import hipann
    import bench
    from ivf_build import build_ivf_list_shard
    from sharded import PartitionedProbes, ShardedSearch, merge_packed_device_torch

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, d, nq, k = 60_000, 96, 200, 10
    stream = torch.cuda.current_stream().cuda_stream
    xq = bench.uniform_queries(torch, nq, d, dev)
    gen = lambda out, row0: bench.gen_uniform_rows(torch, out, row0, 42)  # noqa: E731
    index, info = build_ivf_list_shard(torch, hipann, gen, n, d, 64, 8, 0, rank, world, dev)
    # the replicated scheme: every rank's own coarse step over the whole batch
    rep = ShardedSearch(lambda q, D, I: index.search_device(nq, q.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream),
                        merge_packed_device_torch(hipann, 0), nq, k, dev)
    D0, I0 = rep.search(xq)
    D0, I0 = D0.clone(), I0.clone()
    torch.cuda.synchronize()
    P0 = index.last_probes(nq)
    pp = PartitionedProbes(lambda qs, out: index.coarse_device(qs.shape[0], qs.data_ptr(), out.data_ptr(), stream),
                           nq, 8, dev)

    def local(q, D, I):
        P = pp.probes(q)
        index.search_probes_device(nq, q.data_ptr(), P.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)

    part = ShardedSearch(local, merge_packed_device_torch(hipann, 0), nq, k, dev)
    D1, I1 = part.search(xq)
    torch.cuda.synchronize()
    P1 = pp.probes(xq).cpu().numpy().copy()
    np.savez(f"{result_path}.{rank}.npz", P0=P0, P1=P1, D0=D0.cpu().numpy(), I0=I0.cpu().numpy(), D1=D1.cpu().numpy(),
             I1=I1.cpu().numpy(), last=index.last_probes(nq))
    dist.barrier()
    index.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_ivf_partitioned_coarse_world2_on_one_device(gpu, tmp_path):
    """list-sharded IVF with the coarse step partitioned over two ranks (hipann_ivf_coarse_device
    on each rank's 100-query slice, one all-gather, hipann_ivf_search_probes_device): the probe lists are bit-identical
    to the replicated coarse step's, and the merged top-k (ids and distances) is identical to the replicated scheme's."""
    import torch.multiprocessing as mp

    res = str(tmp_path / "res")
    mp.spawn(_worker_gpu_partitioned, args=(2, _free_port(), res), nprocs=2, join=True)
    for r in range(2):
        z = np.load(f"{res}.{r}.npz")
        assert np.array_equal(z["P1"], z["P0"])
        assert np.array_equal(z["last"], z["P0"])  # the search ran with those lists
        assert np.array_equal(z["I1"], z["I0"]) and np.array_equal(z["D1"], z["D0"])


# ------------------------------------------------------------------------------------------------
# world-4 list sharding on the C3 headline's own list sizes and probe lists
# ------------------------------------------------------------------------------------------------
C3_LISTS = ROOT / "tests" / "golden" / "c3_lists_10m.npz"


def _worker_c3_world4(rank, world, port, result_path):
    dist = _setup(rank, world, port)
    import torch
    from sharded import PartitionedProbes, assign_lists

    z = np.load(C3_LISTS)
    sizes, probes = z["sizes"].astype(np.int64), z["probes"].astype(np.int64)
    nq, nprobe = probes.shape

    def coarse(qidx, out):  # this rank's slice of the batch: the bench's own probe lists of those queries
        out.copy_(torch.from_numpy(probes[qidx[:, 0].numpy()]))

    pp = PartitionedProbes(coarse, nq, nprobe, "cpu")
    P = pp.probes(torch.arange(nq, dtype=torch.int64)[:, None]).numpy().copy()
    owner = assign_lists(sizes, world)
    mine = np.unique(P[P >= 0])
    mine = mine[owner[mine] == rank]
    row_bytes = 2 * 768 + 4  # the fp16 image + the L2 norm per row (the default scan's algorithmic bytes)
    b = torch.tensor([float(sizes[mine].sum()) * row_bytes], dtype=torch.float64)
    allb = [torch.empty_like(b) for _ in range(world)]
    dist.all_gather(allb, b)
    if rank == 0:
        np.savez(result_path, P=P, per_rank=np.array([float(t.item()) for t in allb]), owner=owner)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.skipif(not C3_LISTS.exists(), reason="C3 list fixture not generated")
def test_c3_list_sharding_gloo_world4_balance(tmp_path):
    """The headline's 1024 list sizes and one 1024-query batch's probe lists (tests/golden/c3_lists_10m.npz, written
    by bench.py's C3 run on the MI355X): four gloo ranks each compute their quarter of the probe lists, one all-gather
    (PartitionedProbes) gives every rank the whole batch's lists, identical to the replicated step, and the
    size-balanced list assignment (assign_lists, = hipann_ivf_create's rule) leaves every rank within 5 % of the mean
    per-rank scan bytes; the ranks' bytes add up to the single-GPU scan's."""
    import torch.multiprocessing as mp

    out = tmp_path / "res.npz"
    mp.spawn(_worker_c3_world4, args=(4, _free_port(), str(out)), nprocs=4, join=True)
    r = np.load(out)
    z = np.load(C3_LISTS)
    sizes, probes = z["sizes"].astype(np.int64), z["probes"].astype(np.int64)
    assert np.array_equal(r["P"], probes)
    per = r["per_rank"]
    total = float(sizes[np.unique(probes[probes >= 0])].sum()) * (2 * 768 + 4)
    assert abs(per.sum() - total) <= 1e-6 * total
    assert per.max() / per.mean() <= 1.05, per / per.mean()
    for w in (2, 8):  # the other scaling points of the bench, same rule (host-side check)
        sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
        from sharded import assign_lists
        own = assign_lists(sizes, w)
        lp = np.unique(probes[probes >= 0])
        pw = np.array([sizes[lp[own[lp] == rr]].sum() for rr in range(w)], np.float64)
        assert pw.max() / pw.mean() <= 1.05, (w, pw / pw.mean())
