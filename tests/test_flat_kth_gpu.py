"""The bounded Flat passes' seed k-th (flat_keys_kth, flat_b16k64.hip) against numpy.

The seed bound T0 = (k-th smallest of each query's S sample keys) widened by the relative 2^-20 margin.  The
kernel narrows the search to the keys at or below the k-th smallest per-thread minimum before bisecting; these
tests pin it bit for bit to numpy's order statistic and to the kernel's own full 32-round bisection, on i.i.d.
keys, heavy ties (the narrowed list overflows and the full bisection runs), negative keys, +inf pads, sample
sizes that are not multiples of 256, and both register depths (S <= 4096: 16 keys per thread; else 64).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expected(keys: np.ndarray, k: int) -> np.ndarray:
    t = np.sort(keys, axis=1)[:, k - 1].astype(np.float32)
    out = np.where(np.isinf(t), t, np.maximum(t * np.float32(1.0 + 2.0 ** -20), t + np.float32(2.0 ** -100)))
    return out.astype(np.float32)


def _run(gpu, keys: np.ndarray, k: int, narrow: int) -> np.ndarray:
    import torch

    nq, S = keys.shape
    dk = torch.from_numpy(np.ascontiguousarray(keys, dtype=np.float32)).cuda()
    db = torch.full((nq,), float("nan"), dtype=torch.float32, device="cuda")
    L = gpu.lib()
    f = L.hipann_debug_flat_keys_kth
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int, C.c_void_p, C.c_int]
    assert f(dk.data_ptr(), S, nq, k, db.data_ptr(), narrow) == 0
    return db.cpu().numpy()


def _case(kind: str, nq: int, S: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if kind == "iid":
        return rng.random((nq, S), dtype=np.float32) * 100.0
    if kind == "signed":  # IP keys (-ip): negative and positive
        return rng.standard_normal((nq, S), dtype=np.float32)
    if kind == "ties":  # few distinct values: the narrowed list overflows, the full bisection finishes
        return rng.integers(0, 3, size=(nq, S)).astype(np.float32)
    if kind == "sorted":  # every thread's minimum in the first registers, adversarial for the narrowing
        return np.sort(rng.random((nq, S), dtype=np.float32), axis=1)
    if kind == "inf":  # most keys +inf: the k-th may be +inf
        x = np.full((nq, S), np.inf, dtype=np.float32)
        x[:, :5] = rng.random((nq, 5), dtype=np.float32)
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("S", [40, 1000, 4096, 4097, 16384])
@pytest.mark.parametrize("kind", ["iid", "signed", "ties", "sorted", "inf"])
@pytest.mark.parametrize("k", [1, 10, 32, 64])
def test_flat_keys_kth_matches_numpy(gpu, S, kind, k):
    if S < k:
        pytest.skip("S < k")
    keys = _case(kind, 33, S, seed=S * 7 + k)
    want = _expected(keys, k)
    got = _run(gpu, keys, k, narrow=1)
    full = _run(gpu, keys, k, narrow=0)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    np.testing.assert_array_equal(full.view(np.uint32), want.view(np.uint32))
