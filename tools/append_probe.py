"""Append-path probe (tuning): an IVF index of N x 768 low-rank rows (nlist 1024) built like bench.py, then
2048-row hipann_ivf_add calls timed alone and paired with the next 1024-query search.  HIPANN_APPEND_PROF=1 prints
the library's per-phase host times."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import hipann  # noqa: E402


class A:
    nq = 1024


def main():
    n = int(os.environ.get("PROBE_N", "2000000"))
    dev = torch.device("cuda", 0)
    index, info, xq, _ = bench.build_ivf(A, torch, hipann, 0, 1, dev, n, 768, 1024, 32, 0, 16, 0.02)
    stream = torch.cuda.current_stream().cuda_stream
    D = torch.empty((1024, 10), device=dev)
    I = torch.empty((1024, 10), device=dev, dtype=torch.int64)
    search = lambda: index.search_device(1024, xq.data_ptr(), 10, D.data_ptr(), I.data_ptr(), stream)  # noqa
    for _ in range(3):
        search()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        search()
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / 10 * 1e3
    res = bench.ivf_append_line(torch, index, xq, 10, 768, 16, 0.02, step)
    print(res, flush=True)


if __name__ == "__main__":
    main()
