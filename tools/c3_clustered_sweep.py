"""Calibrate SURVEY §8(d)'s C3 data model on the GPU: 4096 centres U(-1,1)^768 (seed 7), rows = centre + N(0, σ²I)
(seed 42), queries from the same mixture (seed 4242); the GPU IVF build (k-means++ + 25 Lloyd iterations on a
256·nlist sample, FAISS split_clusters for empty clusters); per σ: list-size max/mean and recall@10 / QPS per nprobe
against exact Flat over the same rows.  One JSON line per σ on stdout.
    python tools/c3_clustered_sweep.py [n] [sigma,sigma,...]
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    sigmas = [float(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.3, 0.5, 0.7, 1.0]
    d, nq, nlist, k = 768, 1024, 1024, 10
    dev = torch.device("cuda", 0)
    gc = torch.Generator(device=dev)
    gc.manual_seed(7)
    centres = (torch.rand((4096, d), generator=gc, device=dev, dtype=torch.float32) * 2 - 1).contiguous()
    stream = torch.cuda.current_stream().cuda_stream
    for sigma in sigmas:
        t0 = time.perf_counter()
        xb = torch.empty((n, d), device=dev, dtype=torch.float32)
        bench.gen_clustered_rows(torch, xb, 0, centres, sigma, 42)
        xq = torch.empty((nq, d), device=dev, dtype=torch.float32)
        bench.gen_clustered_rows(torch, xq, 0, centres, sigma, 4242)
        index, info = build_ivf_shard(torch, hipann, xb, 0, n, nlist, 32, 0, 0, 1, centres_seed=1234)
        del xb
        torch.cuda.empty_cache()
        t_build = time.perf_counter() - t0
        gt = flat_ground_truth(torch, hipann, d, 0, xq, k, n, 0, 1, ivf_info_tensor=index)
        D = torch.empty((nq, k), device=dev, dtype=torch.float32)
        I = torch.empty((nq, k), device=dev, dtype=torch.int64)
        sweep = []
        for nprobe in (1, 2, 4, 8, 16, 32, 64, 128, 256):
            index.nprobe = nprobe
            for _ in range(2):
                index.search_device(nq, xq.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)
            torch.cuda.synchronize()
            reps = 5
            t1 = time.perf_counter()
            for _ in range(reps):
                index.search_device(nq, xq.data_ptr(), k, D.data_ptr(), I.data_ptr(), stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t1) * 1e3 / reps
            rec = bench.recall_at(I.cpu().numpy(), gt, k)
            sweep.append({"nprobe": nprobe, "recall_at_10": round(float(rec), 4), "ms": round(ms, 3),
                          "qps": round(nq / (ms * 1e-3), 1)})
            print(f"sigma {sigma} nprobe {nprobe}: recall {rec:.4f} {ms:.3f} ms", file=sys.stderr, flush=True)
            if rec >= 0.995 and nprobe >= 32:
                break
        sizes = np.diff(index._offsets)
        print(json.dumps({"sigma": sigma, "n": n, "build_s": round(t_build, 1),
                          "list_size_max": int(sizes.max()), "list_size_mean": float(sizes.mean()),
                          "list_size_max_over_mean": round(float(sizes.max() / sizes.mean()), 2),
                          "lists_empty": int((sizes == 0).sum()),
                          "list_size_p50_p90_p99": [int(np.percentile(sizes, p)) for p in (50, 90, 99)],
                          "sweep": sweep}), flush=True)
        index.close()
        del index
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
