"""Flat nq = 1 / 4 latency at 10M x 768 (the extension's per-query call): per-call ms, scan and merge kernel ms."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import hipann  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device("cuda", 0)
xb = torch.empty((n, 768), device=dev)
bench.gen_uniform_rows(torch, xb, 0, 42)
xq = bench.uniform_queries(torch, 1024, 768, dev)
ix = hipann.HipIndexFlatDevice(768, 0, xb.data_ptr(), n, 0)
print(json.dumps(bench.flat_latency(torch, hipann, ix, xb, xq, n, 768, 10, 0)))
for nq in (1, 4, 16):
    ix.set_kernel_timing(True)
    D = torch.empty((nq, 10), device=dev)
    I = torch.empty((nq, 10), device=dev, dtype=torch.int64)
    for _ in range(10):
        ix.search_device(nq, xq.data_ptr(), 10, D.data_ptr(), I.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print(f"nq={nq} scan_ms={ix.kernel_ms(0):.4f} merge_ms={ix.kernel_ms(1):.4f}")
    ix.set_kernel_timing(False)
