"""GPU IVF training through the C ABI (hipann_ivf_train / _device).

The extension trains IndexIVFFlat on the CPU at CREATE INDEX (src/faiss_index.cpp:302-319: the stride sample of
train_sample rows, then faiss_idx->train).  hipann_ivf_train runs that k-means on the GPU; its random draws come
from splitmix64(seed), so its result is pinned to the oracle's restatement (oracle_kmeans_train), whose outputs
on the committed fixtures (tests/golden/ivf_train.npz, make_golden.py) the GPU must reproduce: the same
centroids — every cluster sum is fp64 in row order on both sides — and the same cluster sizes, unless an
assignment tie between two centroids resolved differently (none on these fixtures)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

from _data import check_topk_parity

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLD))
from make_golden import TRAIN_CASES, train_data  # noqa: E402


@pytest.mark.parametrize("case", TRAIN_CASES, ids=[c[0] for c in TRAIN_CASES])
def test_ivf_train_equals_oracle_fixture(gpu, case):
    """Host-pointer API on each fixture: stride sample (l2_rand_stride), 256-per-centroid subsample
    (l2_subsample), FAISS random init and k-means++ init, spherical IP, FAISS's split of emptied clusters
    (l2_rand_split)."""
    name, metric, nlist, ts, niter, seed, init, dup = case
    z = np.load(GOLD / "ivf_train.npz")
    cen, sizes = gpu.ivf_train(train_data(dup), nlist, metric, ts, niter, seed, init)
    assert np.array_equal(sizes, z[name + "_sizes"]), (sizes, z[name + "_sizes"])
    assert np.array_equal(cen, z[name + "_cen"]), float(np.abs(cen - z[name + "_cen"]).max())


def test_ivf_train_device_api_equals_host_api(gpu):
    import torch

    x = train_data(False)
    cen_h, _ = gpu.ivf_train(x, 24, 0, 4000, 10, 77, 1)
    xt = torch.from_numpy(x).cuda()
    ct = torch.empty((24, x.shape[1]), device="cuda", dtype=torch.float32)
    gpu.ivf_train_device(x.shape[1], 24, x.shape[0], xt.data_ptr(), ct.data_ptr(), 0, 4000, 10, 77, 1, 0,
                         torch.cuda.current_stream().cuda_stream)
    assert np.array_equal(ct.cpu().numpy(), cen_h)


def test_ivf_train_errors(gpu):
    x = train_data(False)
    with pytest.raises(gpu.HipAnnError):
        gpu.ivf_train(x[:10], 24)  # fewer training points than centroids
    with pytest.raises(gpu.HipAnnError):
        gpu.ivf_train(x, 24, init=7)


def test_ivf_train_then_search_pipeline(gpu, oracle):
    """CREATE INDEX on the GPU end to end: train (train_sample 3000), assign + CSR lists, hipann_ivf_create, search;
    the search follows the oracle's IndexIVFFlat restatement on the same centroids and lists."""
    from _data import build_ivf_lists

    x = train_data(False)
    rng = np.random.default_rng(4)
    xq = (x[rng.integers(0, len(x), 50)] + rng.standard_normal((50, x.shape[1])).astype(np.float32) * 0.1)
    xq = np.ascontiguousarray(xq.astype(np.float32))
    cen, _ = gpu.ivf_train(x, 24, 0, 3000, 25, 1234, 1)
    off, ids, codes = build_ivf_lists(x, cen, 0)
    ix = gpu.HipIndexIVFFlat(cen, off, ids, codes, 4, 0)
    D, I = ix.search(xq, 10)
    Do, Io, Po = oracle.ivf_search(cen, off, ids, codes, xq, 10, 4, 0)
    assert np.array_equal(ix.last_probes(len(xq)), Po)
    check_topk_parity(x, xq, D, I, Do, Io, 0)
    ix.close()
