"""One C3-mixture index (4096 centres U(-1,1)^768 + N(0, σ²I)): per IVF form and nprobe, the batch time
and the exact forms' flagged-query count (rerank_fallbacks), plus a kernel trace friendly loop.
    python tools/ivf_clustered_probe.py SIGMA N NPROBE[,NPROBE...] [FORMS]
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import hipann  # noqa: E402
from ivf_build import build_ivf_shard, flat_ground_truth  # noqa: E402


def main():
    sigma = float(sys.argv[1])
    n = int(sys.argv[2])
    nprobes = [int(x) for x in sys.argv[3].split(",")]
    forms = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [6, 5, 3]
    d, nq, nlist, k = 768, 1024, 1024, 10
    dev = torch.device("cuda", 0)
    gc = torch.Generator(device=dev)
    gc.manual_seed(7)
    centres = (torch.rand((4096, d), generator=gc, device=dev, dtype=torch.float32) * 2 - 1).contiguous()
    xb = torch.empty((n, d), device=dev, dtype=torch.float32)
    bench.gen_clustered_rows(torch, xb, 0, centres, sigma, 42)
    xq = torch.empty((nq, d), device=dev, dtype=torch.float32)
    bench.gen_clustered_rows(torch, xq, 0, centres, sigma, 4242)
    index, info = build_ivf_shard(torch, hipann, xb, 0, n, nlist, 32, 0, 0, 1, centres_seed=1234)
    del xb
    torch.cuda.empty_cache()
    gt = flat_ground_truth(torch, hipann, d, 0, xq, k, n, 0, 1, ivf_info_tensor=index)
    stream = torch.cuda.current_stream().cuda_stream
    D = torch.empty((nq, k), device=dev, dtype=torch.float32)
    I = torch.empty((nq, k), device=dev, dtype=torch.int64)
    for nprobe in nprobes:
        index.nprobe = nprobe
        for form in forms:
            index.form = form
            index.search_device(nq, xq.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)
            torch.cuda.synchronize()
            f0 = index.rerank_fallbacks()
            reps = 3
            index.set_kernel_timing(True)
            t0 = time.perf_counter()
            for _ in range(reps):
                index.search_device(nq, xq.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / reps
            kms, mms = index.kernel_ms(0), index.kernel_ms(1)
            index.set_kernel_timing(False)
            fb = (index.rerank_fallbacks() - f0) / reps
            rec = bench.recall_at(I.cpu().numpy(), gt, k)
            print(json.dumps({"sigma": sigma, "n": n, "nprobe": nprobe, "form": form, "ms": round(ms, 3),
                              "scan_ms": round(kms, 3), "rerank_ms": round(mms, 3), "flagged_per_batch": fb,
                              "recall_at_10": round(float(rec), 4), "path": index.last_search_path()}), flush=True)


if __name__ == "__main__":
    main()
