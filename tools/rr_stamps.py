"""Rerank phase timeline (tuning build HIPANN_RR_STAMP=1): an IVF index like bench.py's headline (PROBE_N rows x 768,
nlist 1024, nprobe 32), a few 1024-query searches, then per query the s_memrealtime stamps (100 MHz) of the wide
rerank's phases: entry, slot range known, candidates selected, distances done, order done, written."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "duckdb-annsearch_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import hipann  # noqa: E402


class A:
    nq = 1024


def main():
    n = int(os.environ.get("PROBE_N", "10000000"))
    dev = torch.device("cuda", 0)
    index, info, xq, _ = bench.build_ivf(A, torch, hipann, 0, 1, dev, n, 768, 1024, 32, 0, 16, 0.02)
    stream = torch.cuda.current_stream().cuda_stream
    D = torch.empty((1024, 10), device=dev)
    I = torch.empty((1024, 10), device=dev, dtype=torch.int64)
    for _ in range(5):
        index.search_device(1024, xq.data_ptr(), 10, D.data_ptr(), I.data_ptr(), stream)
    torch.cuda.synchronize()
    lib = hipann.lib()
    fn = lib.hipann_debug_rr_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    fn.restype = C.c_int
    out = np.zeros(1024 * 8, dtype=np.int64)
    assert fn(out.ctypes.data, out.size) == 0, "not a stamp build"
    full = out.reshape(1024, 8).astype(np.float64) / 100.0  # us
    # stamps in time order: entry, slots, loads landed + compaction (6), wave-0 select done (7), selected (2), ...
    st = full[:, [0, 1, 6, 7, 2, 3, 4, 5]]
    t0 = st[:, 0].min()
    st -= t0
    names = ["entry", "slots", "compacted", "wsel", "merged", "distances", "ordered", "written"]
    print("kernel span (us): first entry 0, last write %.1f" % st[:, 7].max())
    print("entry: p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(st[:, 0], [50, 90, 100])))
    for i in range(1, 8):
        dd = st[:, i] - st[:, i - 1]
        print("%-10s dt p10 %.2f p50 %.2f p90 %.2f max %.2f us" % ((names[i],) + tuple(np.percentile(dd, [10, 50, 90, 100]))))
    print("block life (written - entry): p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(st[:, 7] - st[:, 0], [50, 90, 100])))


if __name__ == "__main__":
    main()
