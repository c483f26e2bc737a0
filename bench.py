#!/usr/bin/env python3
"""bench.py — MI355X search backend benchmark (driver contract: one JSON line on rank 0).

Metric (BASELINE.json): queries/s at recall@10 >= 0.95 on synthetic 10M x 768 fp32, batch = 1024
queries, at 1/2/4/8 GPUs.  A "step" = one search of the 1024-query batch against the whole
database (inputs already resident in HBM when the timed region starts).

Workloads (--workload):
  flat  FAISS Flat L2 over 10M x 768 (exact: recall 1.0).  Rows are sharded contiguously over the
        ranks (strong scaling: the 10M database is fixed, each GPU holds 10M/N rows), every rank
        searches its shard (fp32 MFMA GEMM + fused top-k), the per-rank top-k (1024 x 10 x 12 B) is
        all-gathered over RCCL and merged on every rank.
  ivf   FAISS IVFFlat nlist=1024 nprobe=32 over the same 10M x 768 shape, clustered synthetic data
        (the default workload: the fastest configuration meeting recall@10 >= 0.95); lists are
        sharded over the ranks, same allgather + merge.

Launch: python bench.py [--gpus N --steps K --warmup W]  (N>1 under torch.distributed.run).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TF = 157.3  # MI355X_MICROARCH.md: fp32 MFMA = fp32 vector peak
BF16_MFMA_PEAK_TF = 16 * FP32_MFMA_PEAK_TF  # dense bf16 MFMA = 16x the fp32 matrix rate (~2.5 PF)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["flat", "ivf", "diskann"],
                   default=os.environ.get("HIPANN_BENCH_WORKLOAD", "ivf"))
    p.add_argument("--n", type=int, default=None, help="rows (10M; 1M for diskann)")
    p.add_argument("--d", type=int, default=None, help="dimension (768; 1536 for diskann)")
    p.add_argument("--l-search", type=int, default=128, help="diskann L_search")
    p.add_argument("--degree", type=int, default=64, help="diskann graph degree R")
    p.add_argument("--diskann-host-bfs", action="store_true",
                   help="diskann: the reference-shaped host BFS (one id-gather launch per step) instead of the "
                        "GPU-resident traversal")
    p.add_argument("--nq", type=int, default=1024)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--nlist", type=int, default=1024)
    p.add_argument("--nprobe", type=int, default=32)
    p.add_argument("--metric", choices=["l2", "ip"], default="l2")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-alt-forms", action="store_true", help="ivf/flat: skip timing the other distance forms")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU sample duration")
    a = p.parse_args()
    if a.n is None:
        a.n = 1_000_000 if a.workload == "diskann" else 10_000_000
    if a.d is None:
        a.d = 1536 if a.workload == "diskann" else 768
    return a


CHUNK = 125_000  # generation granularity (divides 10M / {1,2,4,8})


def gen_uniform_rows(torch, out, row0, seed):
    """Fill `out` (rows [row0, row0+len)) with U(-1,1) fp32, chunk-seeded so every sharding sees the
    same global matrix."""
    n = out.shape[0]
    r = 0
    while r < n:
        g_row = row0 + r
        chunk = g_row // CHUNK
        off = g_row - chunk * CHUNK
        take = min(CHUNK - off, n - r)
        gen = torch.Generator(device=out.device)
        gen.manual_seed(seed * 1_000_003 + chunk)
        blk = torch.rand((CHUNK, out.shape[1]), generator=gen, device=out.device, dtype=torch.float32)
        out[r:r + take].copy_(blk[off:off + take]).mul_(2.0).sub_(1.0)
        r += take
    return out


def gen_clustered_rows(torch, out, row0, centres, sigma, seed):
    """Rows = centre[assign] + N(0, sigma^2), chunk-seeded (assignment and noise)."""
    n = out.shape[0]
    nc = centres.shape[0]
    r = 0
    while r < n:
        g_row = row0 + r
        chunk = g_row // CHUNK
        off = g_row - chunk * CHUNK
        take = min(CHUNK - off, n - r)
        gen = torch.Generator(device=out.device)
        gen.manual_seed(seed * 1_000_003 + chunk)
        a = torch.randint(0, nc, (CHUNK,), generator=gen, device=out.device)
        noise = torch.randn((CHUNK, out.shape[1]), generator=gen, device=out.device, dtype=torch.float32)
        blk = centres[a].add_(noise.mul_(sigma))
        out[r:r + take].copy_(blk[off:off + take])
        r += take
    return out


def lowrank_basis(torch, r_dim, d, gen):
    """Random r×d matrix with orthonormal rows (QR of a gaussian), scaled so rows of z·B have O(1) entries."""
    g = torch.randn((d, r_dim), generator=gen, device=gen.device)
    q, _ = torch.linalg.qr(g)
    return (q.T.contiguous() * (d / r_dim) ** 0.5 / 3.0).contiguous()


def gen_lowrank_rows(torch, out, row0, basis, eta, seed):
    """Rows = z·B + eta·N(0, I_d), z ~ N(0, I_r): a low-intrinsic-dimension gaussian (chunk-seeded)."""
    n = out.shape[0]
    r_dim, d = basis.shape
    r = 0
    while r < n:
        g_row = row0 + r
        chunk = g_row // CHUNK
        off = g_row - chunk * CHUNK
        take = min(CHUNK - off, n - r)
        gen = torch.Generator(device=out.device)
        gen.manual_seed(seed * 1_000_003 + chunk)
        z = torch.randn((CHUNK, r_dim), generator=gen, device=out.device, dtype=torch.float32)
        noise = torch.randn((CHUNK, d), generator=gen, device=out.device, dtype=torch.float32)
        blk = torch.addmm(noise.mul_(eta), z, basis)
        out[r:r + take].copy_(blk[off:off + take])
        r += take
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import hipann

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if not hipann.is_available():
        raise SystemExit("libhipann.so / HIP device not available")

    n, d, nq, k = args.n, args.d, args.nq, args.k
    metric = 0 if args.metric == "l2" else 1
    if args.workload == "diskann":
        run_diskann(args, torch, dist, hipann, rank, world, dev)
        return
    from sharded import shard_bounds
    lo, hi = shard_bounds(n, rank, world)
    n_local = hi - lo
    stream = torch.cuda.current_stream().cuda_stream

    # ---------------- data (generated on device; never touches the host) ----------------
    t_setup = time.perf_counter()
    gq = torch.Generator(device=dev)
    gq.manual_seed(4242)
    extra = {}
    if args.workload == "flat":
        xb = torch.empty((n_local, d), device=dev, dtype=torch.float32)
        gen_uniform_rows(torch, xb, lo, 42)
        xq = (torch.rand((nq, d), generator=gq, device=dev, dtype=torch.float32) * 2 - 1).contiguous()
        index = hipann.HipIndexFlatDevice(d, metric, xb.data_ptr(), n_local, local_rank, copy=False,
                                          label_offset=lo)
        # batched q·x form (hipann_flat_set_form): 3 = the library default (2-term split-bf16 scan as a
        # filter + exact direct-form rerank); A/B: 0 exact fp32 MFMA, 1 three-term split, 2 two-term split
        index.form = int(os.environ.get("HIPANN_FLAT_FORM", "3"))
        search = index.search_device
        workload = f"FAISS Flat {'L2' if metric == 0 else 'IP'}, {n // 1_000_000}Mx{d} fp32, batch={nq}, k={k}"
    else:
        from ivf_build import build_ivf_shard  # duckdb-annsearch_amd/ivf_build.py
        gc = torch.Generator(device=dev)
        gc.manual_seed(7)
        data_model = os.environ.get("HIPANN_IVF_DATA", "lowrank")
        xb = torch.empty((n_local, d), device=dev, dtype=torch.float32)
        if data_model == "lowrank":
            r_dim = int(os.environ.get("HIPANN_IVF_RANK", "16"))
            eta = float(os.environ.get("HIPANN_IVF_NOISE", "0.02"))
            basis = lowrank_basis(torch, r_dim, d, gc)
            gen_lowrank_rows(torch, xb, lo, basis, eta, 42)
            xq = torch.empty((nq, d), device=dev, dtype=torch.float32)
            gen_lowrank_rows(torch, xq, 0, basis, eta, 4242)
            data_desc = f"low-rank gaussian, intrinsic dim {r_dim}, noise {eta}"
        else:
            n_centres = int(os.environ.get("HIPANN_IVF_CENTRES", "4096"))
            sigma = float(os.environ.get("HIPANN_IVF_SIGMA", "0.35"))
            centres = (torch.rand((n_centres, d), generator=gc, device=dev) * 2 - 1)
            gen_clustered_rows(torch, xb, lo, centres, sigma, 42)
            a = torch.randint(0, n_centres, (nq,), generator=gq, device=dev)
            xq = (centres[a] + torch.randn((nq, d), generator=gq, device=dev) * sigma).contiguous()
            data_desc = f"{n_centres} gaussian centres, sigma={sigma}"
        index, ivf_info = build_ivf_shard(torch, hipann, xb, lo, n, args.nlist, args.nprobe, metric, rank, world,
                                          centres_seed=1234)
        # list-scan form (hipann_ivf_set_form): 5 = the library default (2-term split-bf16 scan as a
        # filter + exact fp32 direct-form rerank); A/B: 0 fp32 MFMA, 3/4 split scans, 1/2 VALU
        index.form = int(os.environ.get("HIPANN_IVF_FORM", "5"))
        del xb  # lists hold a list-ordered copy
        torch.cuda.empty_cache()
        search = index.search_device
        extra.update(ivf_info)
        workload = (f"FAISS IVFFlat nlist={args.nlist} nprobe={args.nprobe}, {n // 1_000_000}Mx{d} fp32 "
                    f"({data_desc}), batch={nq}, k={k}")
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    from sharded import ShardedSearch, merge_topk_device_torch, shard_bounds

    D_loc = torch.empty((nq, k), device=dev, dtype=torch.float32)
    I_loc = torch.empty((nq, k), device=dev, dtype=torch.int64)

    def local_search(q):
        search(nq, q.data_ptr(), k, D_loc.data_ptr(), I_loc.data_ptr(), stream)
        return D_loc, I_loc

    sharded = ShardedSearch(local_search, merge_topk_device_torch(hipann, metric))

    def step():
        return sharded.search(xq)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.workload == "ivf":
        from ivf_build import scan_bytes
        probes = index.last_probes(nq)
        extra["scan_bytes_per_batch_local"] = scan_bytes(index, probes, d)
        extra["distinct_lists_probed"] = int(np.unique(probes[probes >= 0]).size)
        from ivf_build import scan_pairs
        extra["scanned_pairs_per_batch_local"] = scan_pairs(index, probes)
        from ivf_build import scan_group_rows
        extra["group_rows_per_batch_local"] = scan_group_rows(index, probes)
        cnt = np.bincount(probes[probes >= 0].ravel(), minlength=args.nlist)
        extra["probes_per_list_p50_p90_max"] = [int(np.percentile(cnt, 50)), int(np.percentile(cnt, 90)), int(cnt.max())]

    # ---------------- timed region ----------------
    index.set_kernel_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = index.kernel_ms(0)
    merge_ms = index.kernel_ms(1)
    index.set_kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    qps = nq * args.steps / elapsed

    # ---------------- recall (outside the timed region) ----------------
    Dr, Ir = step()
    torch.cuda.synchronize()
    recall = None
    if args.workload == "ivf":
        from ivf_build import flat_ground_truth
        gt = flat_ground_truth(torch, hipann, d, metric, xq, k, n, rank, world, ivf_info_tensor=index)
        if rank == 0 and gt is not None:
            got = Ir.cpu().numpy()
            recall = float(np.mean([len(set(got[i]) & set(gt[i])) / k for i in range(nq)]))
    else:
        recall = 1.0  # exact search (parity tests: ids identical to the FAISS restatement)

    # ---------------- the other fp32-level list-scan forms, same batch (IVF, 1 GPU) ----------------
    alt = None
    if args.workload == "ivf" and world == 1 and not args.no_alt_forms:
        alt = {}
        base_form = index.form
        names = {0: "fp32_mfma (exact fp32 products)", 3: "split3 (3-term bf16 split, 6 products)",
                 5: "split2_exact (default)"}
        for f in (3, 0):
            if f == base_form:
                continue
            index.form = f
            step()
            torch.cuda.synchronize()
            index.set_kernel_timing(True)
            ta = time.perf_counter()
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            el = time.perf_counter() - ta
            kms = index.kernel_ms(0)
            index.set_kernel_timing(False)
            _, Ia = step()
            torch.cuda.synchronize()
            rec = None
            if gt is not None:
                got = Ia.cpu().numpy()
                rec = float(np.mean([len(set(got[i]) & set(gt[i])) / k for i in range(nq)]))
            alt[names[f]] = {"queries_per_s": round(nq * 5 / el, 1), "scan_kernel_ms": round(kms, 3),
                             "recall_at_10": rec}
        index.form = base_form
        extra["rerank_fallbacks_total"] = index.rerank_fallbacks()

    if args.workload == "flat" and world == 1 and not args.no_alt_forms:
        alt = {}
        base_form = index.form
        for f, nm in ((0, "fp32_mfma (exact fp32 products)"), (1, "split3 (3-term bf16 split, 6 products)")):
            if f == base_form:
                continue
            index.form = f
            step()
            torch.cuda.synchronize()
            index.set_kernel_timing(True)
            ta = time.perf_counter()
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            el = time.perf_counter() - ta
            kms = index.kernel_ms(0)
            index.set_kernel_timing(False)
            _, Ia = step()
            torch.cuda.synchronize()
            same = float((Ia == Ir).float().mean().item())
            alt[nm] = {"queries_per_s": round(nq * 3 / el, 1), "kernel_ms": round(kms, 3),
                       "ids_equal_to_reported_form": round(same, 5)}
        index.form = base_form

    # ---------------- roofline of the dominant kernel ----------------
    if args.workload == "flat":
        flops = 2.0 * nq * n_local * d
        fform = index.form
        if fform == 0:
            kname, terms, peak, fdesc = "flat_gemm_topk2", 1, FP32_MFMA_PEAK_TF, "fp32 MFMA (v_mfma_f32_32x32x2_f32)"
        else:
            terms = 6 if fform == 1 else 3
            kname, peak = "flat_gemm_topk_bf", BF16_MFMA_PEAK_TF
            fdesc = (f"bf16 MFMA (v_mfma_f32_32x32x16_bf16) over a {3 if fform == 1 else 2}-term split: "
                     f"{terms} bf16 products per fp32 product")
            if fform == 3:
                fdesc += ("; the scan keeps 16 (IP: 32) per (split, query) as a filter, merge_ms = exact direct-form "
                          "rerank of the 16 + bound check")
        achieved = terms * flops / (kern_ms * 1e-3) / 1e12 if kern_ms > 0 else 0.0
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": None,
                "kernel": kname, "kernel_ms": round(kern_ms, 3), "merge_ms": round(merge_ms, 3),
                "algorithmic": f"{terms} x 2*nq*N_local*d = {terms * flops:.4g} MFMA FLOP per launch",
                "form": fdesc,
                "fp32_equivalent_tflops": round(flops / (kern_ms * 1e-3) / 1e12, 2) if kern_ms > 0 else None}
    else:
        b_alg = extra.get("scan_bytes_per_batch_local", 0.0)
        form = index.form
        kname, fname = {0: ("ivf_scan_mfma", "decomposed, fp32 MFMA"), 1: ("ivf_scan_topk", "direct, VALU"),
                        2: ("ivf_scan_dot", "decomposed, VALU"),
                        3: ("ivf_scan_mfma_bf", "decomposed, bf16 MFMA over a 3-term split (6 products)"),
                        4: ("ivf_scan_mfma_bf", "decomposed, bf16 MFMA over a 2-term split (3 products)"),
                        5: ("ivf_scan_mfma_bf", "bf16 MFMA 2-term split scan as a filter (16 per list) + exact fp32 "
                            "direct-form rerank, bound-checked (merge_ms includes the rerank)")}[form]
        fpp = 3.0 if form == 1 else 2.0  # flop per (query, row, dim): sub + fma vs fma
        achieved = b_alg / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kname,
                "kernel_ms": round(kern_ms, 3), "merge_ms": round(merge_ms, 3),
                "algorithmic": "sum over distinct probed lists |l|*(4d+8) B per launch",
                "form": fname,
                "scan_tflops": round(fpp * d * extra.get("scanned_pairs_per_batch_local", 0) / (kern_ms * 1e-3) / 1e12, 2)
                if kern_ms > 0 else None}

    tb, tsrc = pmc_traffic(args.workload, roof["kernel"])
    if tb is not None and world == 1:
        roof["traffic"] = round(tb / 1e9, 3)
        roof["traffic_unit"] = "GB per launch (PMC FETCH_SIZE x1024 x2, gfx950 correction)"
        roof["traffic_source"] = tsrc
        roof["algorithmic_per_launch"] = round((b_alg if args.workload == "ivf" else 4.0 * n_local * d) / 1e9, 3)

    # ---------------- CPU baseline (rank 0, N=1 only) ----------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, torch, xq, index, extra, n, d, k, metric)
        except Exception as e:  # report, never fail the bench line
            log(f"[bench] cpu baseline failed: {e!r}")
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        line = {
            "metric": "queries/sec @ recall@10>=0.95, 10Mx768 fp32, batch=1024",
            "value": round(qps, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (generated on device: U(-1,1) rows for flat; low-intrinsic-dimension gaussian rows for ivf)",
            "config": {"workload": workload, "global_batch": nq, "n": n, "d": d, "k": k,
                       "parallelism": f"shard{world}"},
            "recall_at_10": recall,
            "roofline": roof,
            "cpu_baseline": cpu,
            "setup_s": round(setup_s, 1),
        }
        if extra:
            line["ivf"] = {kk: v for kk, v in extra.items() if kk != "scan_bytes_per_batch_local"}
        if alt:
            line["ivf_other_forms" if args.workload == "ivf" else "flat_other_forms"] = alt
        if args.workload == "flat" and index.form == 3:
            line["precision"] = ("returned distances are fp32 direct-form Σ(q−x)² of the returned rows; the bf16 2-term "
                                 "split scan only prunes, and a per-query bound (|scan key − exact| ≤ "
                                 "2^-12·(|q|²+max|x|²)) proves no pruned row reaches the top-k (failures re-run on the "
                                 "3-term path)")
            line["flat"] = {"rerank_fallbacks_total": index.rerank_fallbacks()}
        if args.workload == "ivf" and index.form == 5:
            line["precision"] = ("returned distances are fp32 direct-form Σ(q−x)² (FAISS CPU IVFFlatScanner arithmetic); "
                                 "the bf16 2-term split scan only prunes, and a per-query bound "
                                 "(|scan key − exact| ≤ 2^-12·(|q|²+max|x|²)) proves no pruned row reaches the top-k "
                                 "(failures re-run on the 3-term path)")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_diskann(args, torch, dist, hipann, rank, world, dev):
    """C4: DiskProvider::search_batch over 1M x 1536 SQ8, L_search=128, R=64, nq=1024.

    Graph traversal does not shard, so N GPUs run N replicas (each holds the whole SQ8 DB and answers
    its own 1024-query batch; weak scaling, no collective).  A step = one BFS batch of nq queries:
      * default: diskann_hip_search_batch_resident_device — the traversal on the GPU (one wavefront per
        query, DB + adjacency + visited bitmaps in HBM); roofline of that kernel, algorithmic bytes =
        distances x d (SQ8 code rows) + expansions x 4R (adjacency rows);
      * --diskann-host-bfs: diskann_hip_search_batch — the reference's structure (host lock-step BFS,
        one id-gather launch per step); roofline of the id-gather kernel, d + 12 B per distance
        (code row + id + query_map + out)."""
    import diskann_build as DB

    n, d, nq, k, L, R = args.n, args.d, args.nq, args.k, args.l_search, args.degree
    metric = 0 if args.metric == "l2" else 1
    t_setup = time.perf_counter()
    gc = torch.Generator(device=dev)
    gc.manual_seed(8)
    r_dim = int(os.environ.get("HIPANN_DISKANN_RANK", "16"))
    eta = float(os.environ.get("HIPANN_DISKANN_NOISE", "0.02"))
    basis = lowrank_basis(torch, r_dim, d, gc)
    xb = torch.empty((n, d), device=dev, dtype=torch.float32)
    gen_lowrank_rows(torch, xb, 0, basis, eta, 42)
    xq = torch.empty((nq, d), device=dev, dtype=torch.float32)
    gen_lowrank_rows(torch, xq, 0, basis, eta, 4242 + rank)
    codes, mins, scale = DB.sq8_encode(torch, xb)
    adj_t, medoid = DB.knn_graph(torch, xb, R=R, n_random=R // 4, seed=8)
    torch.cuda.synchronize()
    t_graph = time.perf_counter() - t_setup
    adj = DB.adjacency_u32(torch, adj_t)
    del adj_t
    codes_h = codes.cpu().numpy()
    db = hipann.DiskannDeviceDB(codes_h, hipann.DiskannDeviceDB.FMT_SQ8, mins.cpu().numpy(), scale.cpu().numpy())
    del codes
    torch.cuda.empty_cache()
    xq_h = xq.cpu().numpy()
    eps = np.array([medoid], np.uint32)
    resident = not args.diskann_host_bfs
    stream = torch.cuda.current_stream().cuda_stream
    if resident:
        db.register_graph(adj)
        I_dev = torch.empty((nq, k), device=dev, dtype=torch.int64)
        D_dev = torch.empty((nq, k), device=dev, dtype=torch.float32)
    setup_s = time.perf_counter() - t_setup

    def step():
        if resident:
            st = db.search_batch_resident_device(eps, nq, xq.data_ptr(), k, L, I_dev.data_ptr(), D_dev.data_ptr(),
                                                 metric, stream)
            return None, None, st
        return db.search_batch(adj, eps, xq_h, k, L, metric)

    for _ in range(args.warmup):
        step()
    db.set_kernel_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evals = pops = requeries = 0
    bfs_steps = []
    for _ in range(args.steps):
        ids, dd, st = step()
        evals += st["evals"]
        pops += st.get("pops", 0)
        requeries += st.get("host_requeries", 0)
        bfs_steps.append(st["steps"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_total_ms, launches = db.kernel_stats()
    db.set_kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    qps = world * nq * args.steps / elapsed
    if resident:
        ids = I_dev.cpu().numpy()

    gt = DB.exact_topk(torch, xb, xq, k, metric).cpu().numpy()
    recall = float(np.mean([len(set(ids[i]) & set(gt[i])) / k for i in range(nq)]))
    if resident:
        # per distance: the SQ8 code row (d B); per expansion: the adjacency row (4R B)
        b_alg = evals * d + pops * 4 * R
        achieved = b_alg / (kern_total_ms * 1e-3) / 1e9 if kern_total_ms > 0 else 0.0
        kname = "diskann_bfs"
        alg = (f"distances x d B (SQ8 code rows) + expansions x 4R B (adjacency rows) = "
               f"{b_alg / args.steps / 1e9:.3f} GB per batch (one launch per batch)")
    else:
        b_alg = evals * (d + 12)
        achieved = b_alg / (kern_total_ms * 1e-3) / 1e9 if kern_total_ms > 0 else 0.0
        kname = "dist_ids_sq8"
        alg = (f"distances x (d + 12) B = {d + 12} B per distance (SQ8 code row + id + query_map + out), summed "
               f"over the timed launches")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kname,
            "kernel_ms_per_launch": round(kern_total_ms / max(launches, 1), 4),
            "kernel_ms_per_batch": round(kern_total_ms / args.steps, 3),
            "launches_per_batch": launches / args.steps,
            "distances_per_batch": evals // args.steps,
            "expansions_per_batch": pops // args.steps if resident else None,
            "algorithmic": alg}
    tb, tsrc = pmc_traffic("diskann", kname)
    if tb is not None and world == 1:
        roof["traffic"] = round(tb / 1e9, 4)
        roof["traffic_unit"] = "GB per launch (PMC FETCH_SIZE)"
        roof["traffic_source"] = tsrc

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            from oracle import oracle as O
            c_h = codes_h
            m_h, s_h = mins.cpu().numpy(), scale.cpu().numpy()
            s0 = 16
            t1 = time.perf_counter()
            O.diskann_search_batch(adj, eps, xq_h[:s0], k, L, metric, codes=c_h, mins=m_h, scale=s_h)
            dt0 = time.perf_counter() - t1
            s1 = int(min(nq, max(s0, s0 * args.cpu_seconds / max(dt0, 1e-3))))
            t1 = time.perf_counter()
            O.diskann_search_batch(adj, eps, xq_h[:s1], k, L, metric, codes=c_h, mins=m_h, scale=s_h)
            dt = time.perf_counter() - t1
            cpu = {"value": round(s1 / dt, 2), "unit": "queries/s", "cores": O.num_threads(), "kind": "port",
                   "sample": f"first {s1} of {nq} queries ({dt:.1f} s) through the C oracle's "
                             f"DiskProvider::search_batch restatement (lock-step BFS on the host, SQ8 "
                             f"distances OpenMP over each step's candidates) on the same graph and codes"}
        except Exception as e:
            log(f"[bench] cpu baseline failed: {e!r}")
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        line = {
            "metric": "queries/sec @ recall@10>=0.95 (DiskANN DiskProvider batch path, 1Mx1536 sq8, L_search=128)",
            "value": round(qps, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8 codes, f32 accumulate",
            "data": f"synthetic (generated on device: low-rank gaussian rows, intrinsic dim {r_dim}, noise {eta}; "
                    f"SQ8-encoded; graph = {R - R // 4} exact cell-local nearest neighbours + {R // 4} random "
                    f"edges, medoid entry point)",
            "config": {"workload": f"DISKANN DiskProvider batch-distance, {n // 1_000_000}Mx{d} sq8, "
                                   f"L_search={L}, R={R}, batch={nq}, k={k}",
                       "global_batch": nq * world, "n": n, "d": d, "k": k,
                       "parallelism": f"replicas{world}"},
            "recall_at_10": recall,
            "roofline": roof,
            "cpu_baseline": cpu,
            "setup_s": round(setup_s, 1),
            "diskann": {"graph_build_s": round(t_graph, 1), "bfs_steps_per_batch": int(np.mean(bfs_steps)),
                        "traversal": "GPU-resident (one 2-wavefront workgroup per query)" if resident else
                                     f"host lock-step BFS ({os.environ.get('HIPANN_BFS_THREADS', '16')} threads) + "
                                     f"per-step id-gather launches",
                        "host_requeries": requeries},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(workload: str, kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed FETCH_SIZE pass
    (profiles/rNN/pmc_<workload>.json, written by tools/pmc_traffic.py from a separate
    `rocprofv3 --pmc FETCH_SIZE` run of this same command), or None."""
    for f in sorted((ROOT / "profiles").glob(f"r*/pmc_{workload}.json"), reverse=True):
        try:
            js = json.loads(f.read_text())
        except Exception:
            continue
        if js.get("kernel") == kernel:
            return js.get("hbm_bytes_per_launch"), str(f.relative_to(ROOT))
    return None, None


def cpu_baseline(args, torch, xq, index, extra, n, d, k, metric):
    from oracle import cpu_baseline as CB

    if args.workload == "flat":
        # calibrate on a small slice, then size the sample to ~cpu_seconds (bounded)
        xq_h = xq.cpu().numpy()
        gen_rows = lambda rows: gen_uniform_rows(torch, torch.empty((rows, d), device=xq.device), 0, 42).cpu().numpy()
        probe = gen_rows(20_000)
        q0, dt0, nth = CB.flat_blas_qps(probe, xq_h, k, n, metric)
        rows = int(min(2_000_000, max(20_000, 20_000 * args.cpu_seconds / max(dt0, 1e-3))))
        sample = gen_rows(rows)
        qps, dt, nth = CB.flat_blas_qps(sample, xq_h, k, n, metric)
        return {"value": round(qps, 2), "unit": "queries/s", "cores": nth, "kind": "port",
                "sample": f"all {xq_h.shape[0]} queries x first {rows} of {n} rows ({dt:.1f} s), FAISS "
                          f"BLAS-path restatement (torch CPU sgemm 4096x1024 blocks + norms + top-k), "
                          f"extrapolated linearly to {n} rows"}
    # IVF: the C oracle's IndexIVFFlat::search (OpenMP over queries) on a bounded query subset
    cen, codes, ids = index._keep
    cen_h = cen.cpu().numpy()
    codes_h = codes.cpu().numpy()
    ids_h = ids.cpu().numpy()
    off = index._offsets
    xq_h = xq.cpu().numpy()
    s0 = min(16, xq_h.shape[0])
    _, dt0, nth = CB.ivf_qps(cen_h, off, ids_h, codes_h, xq_h[:s0], k, args.nprobe, metric)
    s = int(min(xq_h.shape[0], max(s0, s0 * args.cpu_seconds / max(dt0, 1e-3))))
    qps, dt, nth = CB.ivf_qps(cen_h, off, ids_h, codes_h, xq_h[:s], k, args.nprobe, metric)
    return {"value": round(qps, 2), "unit": "queries/s", "cores": nth, "kind": "port",
            "sample": f"first {s} of {xq_h.shape[0]} queries ({dt:.1f} s) through the C oracle's FAISS "
                      f"IndexIVFFlat::search restatement (coarse quantizer + direct SIMD distances + heaps, "
                      f"OpenMP over queries) on the same centroids and lists"}


if __name__ == "__main__":
    main()
