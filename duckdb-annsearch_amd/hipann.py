"""hipann — Python host mirror of the extension's GPU search surface, over libhipann.so (C ABI).

This module mirrors, name for name, the reference interfaces that the MI355X backend replaces, so
that tests read like the reference's own tests:

* ``GpuBackend`` / ``get_gpu_backend()`` — src/include/gpu_backend.hpp:12-33 (IsAvailable,
  DeviceInfo, BackendName, CpuToGpu, GpuToCpu) and the link-time singleton ``GetGpuBackend()``.
* ``HipIndexFlat`` — faiss-metal's MetalIndexFlat (faiss-metal/include/faiss-metal/MetalIndexFlat.h):
  ``add``, ``search(n, x, k) -> (D, I)``, ``reconstruct``, ``reset``, ``ntotal``.
* ``HipIndexIVFFlat`` — MetalIndexIVFFlat (faiss-metal/include/faiss-metal/MetalIndexIVFFlat.h).
* ``diskann_*`` — the 3-symbol bridge (src/include/metal_diskann_bridge.h:8-23) and the Rust
  wrappers of rust_lib/src/metal_ffi.rs:33-141 (availability cache, MIN_GPU_WORK gate, bool result).

There is no CPU fallback here: every compute call goes to libhipann.so and raises ``HipAnnError`` when
the library or the device is missing.  The extension's CPU path (FAISS CPU) is not part of this
package; tests use ``oracle/`` as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading
from pathlib import Path
from typing import Optional, Sequence, Tuple

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["HIPANN_LIB"]) if os.environ.get("HIPANN_LIB") else HERE / "libhipann.so"  # override: tuning builds

METRIC_L2 = 0
METRIC_INNER_PRODUCT = 1
MAX_K = 2048

# rust_lib/src/metal_ffi.rs:41, :46 — gates for the DiskANN bridge, from the MI355X break-even measured by
# bench.py (reference_readme_batch_distances, profiles/r02/): against the SIMD CPU distances of the Rust
# caller (n*d ~0.7M) and against the scalar ComputeDistancesCPU of vector_distances (n*d ~65K).
MIN_GPU_WORK = 786432
MIN_GPU_WORK_ONESHOT = 65536
# hip_ann.h HIPANN_AUTO_MIN_WORK: EnsureGpuIndex's AUTO gate on MI355X, ntotal * d (bench.py flat_auto_gate)
AUTO_MIN_WORK = 1048576


class HipAnnError(RuntimeError):
    """Raised when libhipann.so reports an error (the C ABI's err_buf text)."""


_lib = None
_lib_lock = threading.Lock()


def build(force: bool = False) -> Path:
    """Compile libhipann.so for gfx950 (hipcc; no GPU needed)."""
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(HERE / "csrc"), "-j8"], check=True)
    return LIB_PATH


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7,
    but its libc10_hip NEEDs the unversioned name); if libhipann.so were loaded first, torch would map
    a second runtime and see no GPU.  Importing torch first makes libhipann.so bind to torch's copy,
    so device pointers and streams are shared.  Set HIPANN_STANDALONE=1 to skip (no torch use)."""
    if os.environ.get("HIPANN_STANDALONE") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib() -> C.CDLL:
    """Load libhipann.so (fails loudly if it is missing — no fallback)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise HipAnnError(f"libhipann.so not built ({LIB_PATH}); run hipann.build()")
        _share_torch_hip_runtime()
        L = C.CDLL(str(LIB_PATH))
        vp, f, i64p, i64, i32, cp = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int64), C.c_int64, C.c_int, C.c_char_p
        u32p = C.POINTER(C.c_uint32)
        sig = {
            "hipann_available": ([], i32),
            "hipann_device_count": ([], i32),
            "hipann_device_info": ([cp, i32], i32),
            "hipann_peer_access": ([vp, C.POINTER(C.c_int), i32, cp, i32], i32),
            "hipann_flat_create": ([i32, i32, f, i64, C.POINTER(C.c_int), i32, cp, i32], vp),
            "hipann_flat_add": ([vp, f, i64, cp, i32], i32),
            "hipann_flat_search": ([vp, i64, f, i64, f, i64p, cp, i32], i32),
            "hipann_flat_reconstruct": ([vp, i64, f, cp, i32], i32),
            "hipann_flat_create_device": ([i32, i32, vp, i64, i32, i32, i64, cp, i32], vp),
            "hipann_flat_search_device": ([vp, i64, vp, i64, vp, vp, vp, cp, i32], i32),
            "hipann_flat_set_form": ([vp, i32], i32),
            "hipann_flat_get_form": ([vp], i32),
            "hipann_last_search_path": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)], i32),
            "hipann_flat_rerank_fallbacks": ([vp], i64),
            "hipann_flat_host_syncs": ([vp], i64),
            "hipann_merge_topk_device": ([i32, i32, i64, i64, vp, vp, vp, vp, vp, cp, i32], i32),
            "hipann_merge_topk_packed_device": ([i32, i32, i64, i64, vp, i64, vp, vp, vp, cp, i32], i32),
            "hipann_ivf_create": ([i32, i32, i32, i32, f, i64p, i64p, f, C.POINTER(C.c_int), i32, cp, i32], vp),
            "hipann_ivf_create_device": ([i32, i32, i32, i32, vp, i64p, vp, vp, i32, i32, cp, i32], vp),
            "hipann_ivf_search": ([vp, i64, f, i64, f, i64p, cp, i32], i32),
            "hipann_ivf_search_device": ([vp, i64, vp, i64, vp, vp, vp, cp, i32], i32),
            "hipann_ivf_coarse_device": ([vp, i64, vp, vp, vp, cp, i32], i32),
            "hipann_ivf_search_probes_device": ([vp, i64, vp, vp, i64, vp, vp, vp, cp, i32], i32),
            "hipann_ivf_last_probes": ([vp, i64p, i64, cp, i32], i32),
            "hipann_ivf_set_nprobe": ([vp, i32], i32),
            "hipann_ivf_get_nprobe": ([vp], i32),
            "hipann_ivf_nlist": ([vp], i32),
            "hipann_ivf_search_np": ([vp, i32, i64, f, i64, f, i64p, cp, i32], i32),
            "hipann_ivf_add": ([vp, i64, f, i64p, cp, i32], i32),
            "hipann_ivf_export": ([vp, f, i64p, i64p, f, cp, i32], i32),
            "hipann_ivf_train": ([i32, i32, i32, i64, f, i64, i32, C.c_uint64, i32, i32, f, i64p, cp, i32], i32),
            "hipann_ivf_train_device": ([i32, i32, i32, i64, vp, i64, i32, C.c_uint64, i32, i32, vp, vp, cp, i32],
                                        i32),
            "hipann_flat_reconstruct_n": ([vp, i64, i64, f, cp, i32], i32),
            "hipann_ivf_set_form": ([vp, i32], i32),
            "hipann_ivf_get_form": ([vp], i32),
            "hipann_ivf_rerank_fallbacks": ([vp], i64),
            "hipann_ntotal": ([vp], i64),
            "hipann_dim": ([vp], i32),
            "hipann_metric": ([vp], i32),
            "hipann_memory_bytes": ([vp], i64),
            "hipann_free": ([vp], None),
            "hipann_set_kernel_timing": ([vp, i32], i32),
            "hipann_last_kernel_ms": ([vp, i32], C.c_double),
            "diskann_hip_available": ([], i32),
            "diskann_hip_batch_distances": ([f, f, i32, i32, i32, f], i32),
            "diskann_hip_multi_batch_distances": ([f, f, u32p, i32, i32, i32, i32, f], i32),
            "diskann_metal_available": ([], i32),
            "diskann_metal_batch_distances": ([f, f, i32, i32, i32, f], i32),
            "diskann_metal_multi_batch_distances": ([f, f, u32p, i32, i32, i32, i32, f], i32),
            "diskann_hip_register_db": ([vp, i64, i32, i32, f, f], vp),
            "diskann_hip_multi_batch_distances_ids": ([vp, f, i32, u32p, u32p, i32, i32, f], i32),
            "diskann_hip_multi_batch_distances_ids_device": ([vp, vp, i32, vp, vp, i32, i32, vp, vp], i32),
            "diskann_hip_db_size": ([vp], i64),
            "diskann_hip_release_db": ([vp], None),
            "diskann_hip_set_kernel_timing": ([vp, i32], i32),
            "diskann_hip_register_graph": ([vp, C.POINTER(C.c_uint32), i32], i32),
            "diskann_hip_search_batch_resident": ([vp, C.POINTER(C.c_uint32), i32, f, i32, i32, i32, i32, i64p, f,
                                                   i64p, cp, i32], i32),
            "diskann_hip_search_batch_resident_device": ([vp, C.POINTER(C.c_uint32), i32, vp, i32, i32, i32, i32, vp,
                                                          vp, i64p, vp, cp, i32], i32),
            "diskann_hip_kernel_stats": ([vp, C.POINTER(C.c_double), i64p], i32),
            "diskann_hip_search_batch": ([vp, C.POINTER(C.c_uint32), i32, C.POINTER(C.c_uint32), i32, f, i32, i32,
                                          i32, i32, i64p, f, i64p, cp, i32], i32),
        }
        missing = [name for name in sig if not hasattr(L, name)]
        if missing:
            raise HipAnnError(f"libhipann.so is missing exports: {missing}")
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
        return L


def _ptr(a: Optional[np.ndarray], t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def _err() -> C.Array:
    return C.create_string_buffer(1024)


def _check(rc, eb) -> None:
    if rc != 0:
        raise HipAnnError(eb.value.decode(errors="replace") or "hipann error")


def _f32_2d(x, d: Optional[int] = None) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x.reshape(1, -1) if d is None else x.reshape(-1, d)
    if d is not None and x.shape[1] != d:
        raise ValueError(f"expected dimension {d}, got {x.shape[1]}")
    return x


def is_available() -> bool:
    try:
        return bool(lib().hipann_available())
    except (HipAnnError, OSError):
        return False


def device_count() -> int:
    return int(lib().hipann_device_count())


def device_info() -> str:
    buf = C.create_string_buffer(512)
    lib().hipann_device_info(buf, 512)
    return buf.value.decode()


# ------------------------------------------------------------------------------------------------
# Index handles
# ------------------------------------------------------------------------------------------------
class _Handle:
    def __init__(self, h, d: int, metric: int):
        if not h:
            raise HipAnnError("null handle")
        self._h = C.c_void_p(h)
        self.d = d
        self.metric_type = metric

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().hipann_free(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    @property
    def ntotal(self) -> int:
        return int(lib().hipann_ntotal(self._h))

    @property
    def memory_bytes(self) -> int:
        return int(lib().hipann_memory_bytes(self._h))

    def set_kernel_timing(self, on: bool) -> None:
        lib().hipann_set_kernel_timing(self._h, 1 if on else 0)

    def last_search_path(self) -> dict:
        """hipann_last_search_path: the form the last search's scan ran, its rerank filter depth (0 = none) and
        the IVF sub-lists per slot (0 = merged lists)."""
        f, kf, sl = C.c_int(-1), C.c_int(0), C.c_int(0)
        lib().hipann_last_search_path(self._h, C.byref(f), C.byref(kf), C.byref(sl))
        return {"form": f.value, "filter_k": kf.value, "sublists": sl.value}

    def kernel_ms(self, which: int = 0) -> float:
        return float(lib().hipann_last_kernel_ms(self._h, which))

    PEER_SAME_DEVICE, PEER_ENABLED, PEER_UNAVAILABLE = 2, 1, 0

    def peer_access(self) -> list:
        """hipann_peer_access: per shard, 2 = on the first shard's device, 1 = peer access enabled both ways with it
        (the top-k gather rides xGMI), 0 = not available (the gather stages through host memory)."""
        eb = _err()
        n = lib().hipann_peer_access(self._h, None, 0, eb, 1024)
        _check(min(n, 0), eb)
        st = (C.c_int * max(n, 1))()
        _check(min(lib().hipann_peer_access(self._h, st, n, eb, 1024), 0), eb)
        return [int(st[i]) for i in range(n)]

    @property
    def handle(self) -> C.c_void_p:
        return self._h


class _FlatForm:
    """q·x form of the batched (nq >= 20) Flat path — hipann_flat_set_form (hip_ann.h)."""

    FORM_FP32 = 0          # exact fp32 products on the fp32 matrix cores
    FORM_SPLIT3 = 1        # 3-term split-bf16 products (fp32-level) on the bf16 matrix cores
    FORM_SPLIT2 = 2        # 2-term split (~2^-16 relative per product; measurement only)
    FORM_SPLIT2_EXACT = 3  # the 2-term scan as a filter + exact direct-form rerank with a bound check
    FORM_BF16_EXACT = 4    # one bf16 product per element (tiled bf16 image) as the filter, same rerank
    FORM_I8_EXACT = 5      # default (bounded passes: nq >= 256, >= 512K rows, d <= 1024; else form 4): one int8 product per element (tiled int8 image, int32 sums) as the filter, same rerank

    @property
    def form(self) -> int:
        return int(lib().hipann_flat_get_form(self._h))

    @form.setter
    def form(self, v: int) -> None:
        if lib().hipann_flat_set_form(self._h, int(v)) != 0:
            raise HipAnnError("form must be 0 (fp32), 1 (split bf16, 3 terms), 2 (split bf16, 2 terms), "
                              "3 (split bf16 + exact rerank), 4 (bf16 + exact rerank) or 5 (int8 + exact rerank)")

    def rerank_fallbacks(self) -> int:
        """Queries the exact form's bound check re-ran on the 3-term path since creation."""
        return int(lib().hipann_flat_rerank_fallbacks(self._h))

    def host_syncs(self) -> int:
        """Host synchronisations made by this index's searches since creation (hipann_flat_host_syncs)."""
        return int(lib().hipann_flat_host_syncs(self._h))


class HipIndexFlat(_FlatForm, _Handle):
    """Flat index on MI355X — MetalIndexFlat's API (MetalIndexFlat.h:45-101)."""

    def __init__(self, d: int, metric: int = METRIC_L2, xb=None, devices: Optional[Sequence[int]] = None):
        x = _f32_2d(xb, d) if xb is not None else np.zeros((0, d), np.float32)
        devs = (C.c_int * len(devices))(*devices) if devices else None
        eb = _err()
        h = lib().hipann_flat_create(d, metric, _ptr(x, C.c_float), x.shape[0], devs, len(devices) if devices else 0,
                                     eb, 1024)
        if not h:
            raise HipAnnError(eb.value.decode())
        super().__init__(h, d, metric)

    def add(self, x) -> None:
        x = _f32_2d(x, self.d)
        eb = _err()
        _check(lib().hipann_flat_add(self._h, _ptr(x, C.c_float), x.shape[0], eb, 1024), eb)

    def search(self, x, k: int) -> Tuple[np.ndarray, np.ndarray]:
        x = _f32_2d(x, self.d)
        n = x.shape[0]
        D = np.empty((n, max(k, 0)), np.float32)
        I = np.empty((n, max(k, 0)), np.int64)
        eb = _err()
        _check(lib().hipann_flat_search(self._h, n, _ptr(x, C.c_float), k, _ptr(D, C.c_float), _ptr(I, C.c_int64),
                                        eb, 1024), eb)
        return D, I

    def reconstruct_n(self, i0: int, n: int) -> np.ndarray:
        """faiss::Index::reconstruct_n: rows [i0, i0 + n) back to host in one call."""
        out = np.empty((max(n, 0), self.d), np.float32)
        eb = _err()
        _check(lib().hipann_flat_reconstruct_n(self._h, i0, n, _ptr(out, C.c_float), eb, 1024), eb)
        return out

    def reconstruct(self, key: int) -> np.ndarray:
        out = np.empty(self.d, np.float32)
        eb = _err()
        _check(lib().hipann_flat_reconstruct(self._h, key, _ptr(out, C.c_float), eb, 1024), eb)
        return out


class HipIndexFlatDevice(_FlatForm, _Handle):
    """Flat shard over an HBM-resident matrix (torch CUDA tensor or raw pointer) — the sharded /
    benchmark path.  ``search_device`` is asynchronous on ``stream``."""

    def __init__(self, d: int, metric: int, xb_ptr: int, n: int, device: int = 0, copy: bool = False,
                 label_offset: int = 0):
        eb = _err()
        h = lib().hipann_flat_create_device(d, metric, C.c_void_p(xb_ptr), n, device, 1 if copy else 0, label_offset,
                                            eb, 1024)
        if not h:
            raise HipAnnError(eb.value.decode())
        super().__init__(h, d, metric)

    def search_device(self, nq: int, xq_ptr: int, k: int, d_ptr: int, i_ptr: int, stream: int = 0) -> None:
        eb = _err()
        _check(lib().hipann_flat_search_device(self._h, nq, C.c_void_p(xq_ptr), k, C.c_void_p(d_ptr),
                                               C.c_void_p(i_ptr), C.c_void_p(stream or None), eb, 1024), eb)


def merge_topk_device(metric: int, nparts: int, nq: int, k: int, d_parts: int, i_parts: int, d_out: int, i_out: int,
                      stream: int = 0) -> None:
    """Merge [part][nq][k] partial results (device pointers) — after the RCCL allgather."""
    eb = _err()
    _check(lib().hipann_merge_topk_device(metric, nparts, nq, k, C.c_void_p(d_parts), C.c_void_p(i_parts),
                                          C.c_void_p(d_out), C.c_void_p(i_out), C.c_void_p(stream or None), eb, 1024),
           eb)


def merge_topk_packed_device(metric: int, nparts: int, nq: int, k: int, parts: int, part_bytes: int, d_out: int,
                             i_out: int, stream: int = 0) -> None:
    """hipann_merge_topk_packed_device: merge of the all-gathered packed parts ([labels int64 nq·k]
    [distances fp32 nq·k] per part, part_bytes apart) — sharded.py's single-collective layout."""
    eb = _err()
    _check(lib().hipann_merge_topk_packed_device(metric, nparts, nq, k, C.c_void_p(parts), part_bytes,
                                                 C.c_void_p(d_out), C.c_void_p(i_out), C.c_void_p(stream or None), eb,
                                                 1024), eb)


class HipIndexIVFFlat(_Handle):
    """IVFFlat on MI355X — MetalIndexIVFFlat's API (MetalIndexIVFFlat.h:12-76).  Built from a trained
    coarse quantizer (centroids) and CSR inverted lists, as index_cpu_to_metal_ivf copies them out of
    a FAISS IndexIVFFlat (MetalIndexIVFFlat.mm:283-326)."""

    def __init__(self, centroids, list_offsets, ids, codes, nprobe: int = 1, metric: int = METRIC_L2,
                 devices: Optional[Sequence[int]] = None):
        cen = _f32_2d(centroids)
        nlist, d = cen.shape
        off = np.ascontiguousarray(list_offsets, np.int64)
        idv = np.ascontiguousarray(ids, np.int64)
        cod = _f32_2d(codes, d) if len(idv) else np.zeros((0, d), np.float32)
        if off.shape != (nlist + 1,) or off[-1] != len(idv) or cod.shape[0] != len(idv):
            raise ValueError("inconsistent inverted lists")
        devs = (C.c_int * len(devices))(*devices) if devices else None
        eb = _err()
        h = lib().hipann_ivf_create(d, metric, nlist, nprobe, _ptr(cen, C.c_float), _ptr(off, C.c_int64),
                                    _ptr(idv, C.c_int64), _ptr(cod, C.c_float), devs,
                                    len(devices) if devices else 0, eb, 1024)
        if not h:
            raise HipAnnError(eb.value.decode())
        super().__init__(h, d, metric)
        self.nlist = nlist
        self._nprobe = nprobe

    @classmethod
    def from_device(cls, d: int, metric: int, nlist: int, nprobe: int, centroids_ptr: int, list_offsets,
                    ids_ptr: int, codes_ptr: int, device: int = 0, copy: bool = False) -> "HipIndexIVFFlat":
        off = np.ascontiguousarray(list_offsets, np.int64)
        eb = _err()
        h = lib().hipann_ivf_create_device(d, metric, nlist, nprobe, C.c_void_p(centroids_ptr), _ptr(off, C.c_int64),
                                           C.c_void_p(ids_ptr), C.c_void_p(codes_ptr), device, 1 if copy else 0, eb,
                                           1024)
        if not h:
            raise HipAnnError(eb.value.decode())
        obj = cls.__new__(cls)
        _Handle.__init__(obj, h, d, metric)
        obj.nlist = nlist
        obj._nprobe = nprobe
        return obj

    @property
    def nprobe(self) -> int:
        return self._nprobe

    @nprobe.setter
    def nprobe(self, v: int) -> None:
        if lib().hipann_ivf_set_nprobe(self._h, int(v)) != 0:
            raise HipAnnError("nprobe must be >= 1")
        self._nprobe = int(v)

    FORM_DECOMPOSED = 0       # ‖q‖² + ‖x‖² − 2 q·x on the fp32 matrix cores (FAISS GPU / faiss-metal IVF form)
    FORM_DIRECT = 1           # Σ(q − x)² (FAISS CPU IndexIVFFlat scanner form)
    FORM_DECOMPOSED_VALU = 2  # the decomposed form on the VALU kernel (A/B measurement)
    FORM_SPLIT3 = 3           # decomposed, q·x on the bf16 matrix cores over a 3-term bf16 split (6 products)
    FORM_SPLIT2 = 4           # decomposed, 2-term bf16 split (3 products, ~2^-16 relative per product)
    FORM_SPLIT2_EXACT = 5     # the SPLIT2 scan as a filter + exact direct-form rerank with a bound check
    FORM_HALF_EXACT = 6       # default: the same rerank, the filter scan over a tiled fp16 image (half the bytes)
    FORM_I8_EXACT = 7         # opt-in: the same rerank, the filter scan over a tiled int8 image (a quarter of the bytes)

    @property
    def form(self) -> int:
        return int(lib().hipann_ivf_get_form(self._h))

    @form.setter
    def form(self, v: int) -> None:
        if lib().hipann_ivf_set_form(self._h, int(v)) != 0:
            raise HipAnnError("form must be 0 (decomposed), 1 (direct), 2 (decomposed, VALU), 3 or 4 (split bf16), "
                              "5 (split bf16 + exact rerank), 6 (fp16 image + exact rerank), 7 (int8 image + exact rerank)")

    def search(self, x, k: int, nprobe: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """search(n, x, k) — with ``nprobe`` the per-call SearchParametersIVF value (hipann_ivf_search_np:
        read under the handle's lock, the index's own nprobe is left unchanged)."""
        x = _f32_2d(x, self.d)
        n = x.shape[0]
        D = np.empty((n, max(k, 0)), np.float32)
        I = np.empty((n, max(k, 0)), np.int64)
        eb = _err()
        if nprobe is None:
            rc = lib().hipann_ivf_search(self._h, n, _ptr(x, C.c_float), k, _ptr(D, C.c_float), _ptr(I, C.c_int64),
                                         eb, 1024)
        else:
            if int(nprobe) < 1:
                raise HipAnnError("nprobe must be >= 1")
            rc = lib().hipann_ivf_search_np(self._h, int(nprobe), n, _ptr(x, C.c_float), k, _ptr(D, C.c_float),
                                            _ptr(I, C.c_int64), eb, 1024)
        _check(rc, eb)
        return D, I

    def add(self, x, ids=None) -> None:
        """IndexIVFFlat::add / add_with_ids on the GPU copy (hipann_ivf_add): rows assigned by the GPU
        coarse quantizer, appended to their lists in insertion order; labels ``ids`` or ntotal + i."""
        x = _f32_2d(x, self.d)
        idv = None if ids is None else np.ascontiguousarray(ids, np.int64)
        if idv is not None and idv.shape != (x.shape[0],):
            raise ValueError("ids must hold one label per row")
        eb = _err()
        _check(lib().hipann_ivf_add(self._h, x.shape[0], _ptr(x, C.c_float), _ptr(idv, C.c_int64), eb, 1024), eb)

    def export(self) -> dict:
        """The index in FAISS ArrayInvertedLists CSR form (hipann_ivf_export): centroids, list_offsets,
        ids, codes, nprobe, metric — what GpuToCpu rebuilds a CPU IndexIVFFlat from."""
        off = np.empty(self.nlist + 1, np.int64)
        eb = _err()
        _check(lib().hipann_ivf_export(self._h, None, _ptr(off, C.c_int64), None, None, eb, 1024), eb)
        n = int(off[-1])
        cen = np.empty((self.nlist, self.d), np.float32)
        ids = np.empty(n, np.int64)
        codes = np.empty((n, self.d), np.float32)
        _check(lib().hipann_ivf_export(self._h, _ptr(cen, C.c_float), _ptr(off, C.c_int64), _ptr(ids, C.c_int64),
                                       _ptr(codes, C.c_float), eb, 1024), eb)
        return {"type": "IVFFlat", "centroids": cen, "list_offsets": off, "ids": ids, "codes": codes,
                "nprobe": int(lib().hipann_ivf_get_nprobe(self._h)), "metric": self.metric_type}

    def search_device(self, nq: int, xq_ptr: int, k: int, d_ptr: int, i_ptr: int, stream: int = 0) -> None:
        eb = _err()
        _check(lib().hipann_ivf_search_device(self._h, nq, C.c_void_p(xq_ptr), k, C.c_void_p(d_ptr),
                                              C.c_void_p(i_ptr), C.c_void_p(stream or None), eb, 1024), eb)

    def coarse_device(self, nq: int, xq_ptr: int, probes_ptr: int, stream: int = 0) -> None:
        """The coarse step alone (hipann_ivf_coarse_device): nq x min(nprobe, nlist) int64 probe lists."""
        eb = _err()
        _check(lib().hipann_ivf_coarse_device(self._h, nq, C.c_void_p(xq_ptr), C.c_void_p(probes_ptr),
                                              C.c_void_p(stream or None), eb, 1024), eb)

    def search_probes_device(self, nq: int, xq_ptr: int, probes_ptr: int, k: int, d_ptr: int, i_ptr: int,
                             stream: int = 0) -> None:
        """search_device with the caller's probe lists (hipann_ivf_search_probes_device): no coarse step."""
        eb = _err()
        _check(lib().hipann_ivf_search_probes_device(self._h, nq, C.c_void_p(xq_ptr), C.c_void_p(probes_ptr), k,
                                                     C.c_void_p(d_ptr), C.c_void_p(i_ptr), C.c_void_p(stream or None),
                                                     eb, 1024), eb)

    def rerank_fallbacks(self) -> int:
        """Queries the exact form's bound check flagged since creation (re-run on the device in the direct form)."""
        return int(lib().hipann_ivf_rerank_fallbacks(self._h))

    def last_probes(self, nq: int) -> np.ndarray:
        P = np.empty((nq, min(self._nprobe, self.nlist)), np.int64)
        eb = _err()
        _check(lib().hipann_ivf_last_probes(self._h, _ptr(P, C.c_int64), P.size, eb, 1024), eb)
        return P


KMEANS_INIT_RANDOM, KMEANS_INIT_PLUSPLUS = 0, 1


def ivf_train(x, nlist: int, metric: int = METRIC_L2, train_sample: int = 0, niter: int = 25, seed: int = 1234,
              init: int = KMEANS_INIT_PLUSPLUS, device: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """hipann_ivf_train: IndexIVFFlat::train on the GPU (k-means over the stride sample of train_sample rows,
    faiss_index.cpp:302-319).  Returns (centroids nlist x d, the last iteration's cluster sizes)."""
    x = _f32_2d(x)
    n, d = x.shape
    cen = np.empty((nlist, d), np.float32)
    sizes = np.empty(nlist, np.int64)
    eb = _err()
    _check(lib().hipann_ivf_train(d, metric, nlist, n, _ptr(x, C.c_float), train_sample, niter, seed, init, device,
                                  _ptr(cen, C.c_float), _ptr(sizes, C.c_int64), eb, 1024), eb)
    return cen, sizes


def ivf_train_device(d: int, nlist: int, n: int, x_ptr: int, centroids_ptr: int, metric: int = METRIC_L2,
                     train_sample: int = 0, niter: int = 25, seed: int = 1234, init: int = KMEANS_INIT_PLUSPLUS,
                     device: int = 0, stream: int = 0) -> None:
    """hipann_ivf_train_device: the same with the rows (n x d fp32) and the centroids (nlist x d) in HBM."""
    eb = _err()
    _check(lib().hipann_ivf_train_device(d, metric, nlist, n, C.c_void_p(x_ptr), train_sample, niter, seed, init,
                                         device, C.c_void_p(centroids_ptr), C.c_void_p(stream or None), eb, 1024), eb)


# ------------------------------------------------------------------------------------------------
# GpuBackend (src/include/gpu_backend.hpp:12-33) — the drop-in boundary of the FAISS path
# ------------------------------------------------------------------------------------------------
class GpuBackend:
    """HIP implementation of the extension's GpuBackend interface.

    ``cpu_to_gpu`` accepts the pieces of a FAISS CPU index the reference's converters read
    (IndexFlat: d, metric, xb — MetalIndexFlat.mm:504-515; IndexIVFFlat: centroids, inverted
    lists, nprobe — MetalIndexIVFFlat.mm:283-326) as a dict, dispatching IVFFlat first and Flat
    second like MetalGpuBackend::CpuToGpu (gpu_backend_metal.mm:45-60).  Errors raise
    ``RuntimeError`` (the type faiss_index.cpp:122-124 / :146-148 catch).
    """

    def is_available(self) -> bool:
        return is_available()

    def device_info(self) -> str:
        if not self.is_available():
            return "HIP: not available"
        return "HIP GPU (" + device_info() + ")"

    def backend_name(self) -> str:
        return "hip"

    def auto_upload(self, ntotal: int, d: int, index_type: str = "Flat") -> bool:
        """FaissIndex::EnsureGpuIndex's AUTO branch (faiss_index.cpp:128-149) with the MI355X gate: no backend or
        HNSW → CPU; otherwise upload when ntotal * d >= AUTO_MIN_WORK (the Metal gates ntotal >= 256, d >= 128
        upload tables whose per-query GPU call is slower than the CPU scan on this part)."""
        if not self.is_available() or index_type.lower() == "hnsw":
            return False
        return int(ntotal) * int(d) >= AUTO_MIN_WORK

    def cpu_to_gpu(self, cpu_index: dict):
        if not self.is_available():
            raise RuntimeError("HIP GPU backend not available")
        kind = cpu_index.get("type")
        try:
            if kind == "IVFFlat":
                return HipIndexIVFFlat(cpu_index["centroids"], cpu_index["list_offsets"], cpu_index["ids"],
                                       cpu_index["codes"], cpu_index.get("nprobe", 1),
                                       cpu_index.get("metric", METRIC_L2))
            if kind == "Flat":
                return HipIndexFlat(cpu_index["d"], cpu_index.get("metric", METRIC_L2), cpu_index["xb"])
        except HipAnnError as e:
            raise RuntimeError(str(e)) from e
        raise RuntimeError("HIP GPU supports IndexFlat and IndexIVFFlat. Got an unsupported index type.")

    def gpu_to_cpu(self, gpu_index) -> dict:
        if isinstance(gpu_index, HipIndexFlat):
            return {"type": "Flat", "d": gpu_index.d, "metric": gpu_index.metric_type,
                    "xb": gpu_index.reconstruct_n(0, gpu_index.ntotal)}
        if isinstance(gpu_index, HipIndexIVFFlat):  # gpu_backend_metal.mm:62-67 (index_metal_to_cpu_ivf)
            return gpu_index.export()
        raise RuntimeError("Index is not a HIP index -- cannot convert to CPU")


_backend = None


def get_gpu_backend() -> GpuBackend:
    """The process-wide backend singleton (GetGpuBackend(), gpu_backend_metal.mm:81-84)."""
    global _backend
    if _backend is None:
        _backend = GpuBackend()
    return _backend


# ------------------------------------------------------------------------------------------------
# DiskANN bridge (metal_diskann_bridge.h:8-23) + metal_ffi.rs-style wrappers
# ------------------------------------------------------------------------------------------------
_hip_status = -1
_status_lock = threading.Lock()


def diskann_hip_available() -> int:
    return int(lib().diskann_hip_available())


def diskann_hip_batch_distances(query, candidates, n: int, dim: int, metric: int, out: np.ndarray) -> int:
    """Raw C-ABI call (0 / -1), buffers as numpy arrays."""
    q = np.ascontiguousarray(query, np.float32)
    c = np.ascontiguousarray(candidates, np.float32)
    return int(lib().diskann_hip_batch_distances(_ptr(q, C.c_float), _ptr(c, C.c_float), n, dim, metric,
                                                 _ptr(out, C.c_float)))


def diskann_hip_multi_batch_distances(queries, candidates, query_map, total_n: int, nq: int, dim: int, metric: int,
                                      out: np.ndarray) -> int:
    q = np.ascontiguousarray(queries, np.float32)
    c = np.ascontiguousarray(candidates, np.float32)
    m = np.ascontiguousarray(query_map, np.uint32)
    return int(lib().diskann_hip_multi_batch_distances(_ptr(q, C.c_float), _ptr(c, C.c_float), _ptr(m, C.c_uint32),
                                                       total_n, nq, dim, metric, _ptr(out, C.c_float)))


def is_hip_available() -> bool:
    """Cached availability (metal_ffi.rs:33-57 is_metal_available)."""
    global _hip_status
    with _status_lock:
        if _hip_status < 0:
            try:
                _hip_status = 1 if diskann_hip_available() == 1 else 0
            except (HipAnnError, OSError):
                _hip_status = 0
        return _hip_status == 1


def hip_batch_distances(query, candidates, n: int, dim: int, metric: int, out: np.ndarray) -> bool:
    """metal_ffi.rs:67-95 metal_batch_distances: True on success; False when unavailable, below the
    MIN_GPU_WORK gate, or on failure (the caller then computes on the CPU)."""
    if n == 0 or dim == 0:
        return True
    if n * dim < MIN_GPU_WORK or not is_hip_available():
        return False
    return diskann_hip_batch_distances(query, candidates, n, dim, metric, out) == 0


def hip_multi_batch_distances(queries, candidates, query_map, total_n: int, nq: int, dim: int, metric: int,
                              out: np.ndarray) -> bool:
    """metal_ffi.rs:107-141 metal_multi_batch_distances (no MIN_GPU_WORK check; the caller gates)."""
    if total_n == 0 or nq == 0 or dim == 0:
        return True
    if not is_hip_available():
        return False
    return diskann_hip_multi_batch_distances(queries, candidates, query_map, total_n, nq, dim, metric, out) == 0


class DiskannDeviceDB:
    """HBM-resident DiskANN vectors (fp32 or SQ8) + the id-gather distance call."""

    FMT_F32, FMT_SQ8 = 0, 1

    def __init__(self, data: np.ndarray, fmt: int = 0, sq8_min=None, sq8_scale=None):
        if fmt == self.FMT_F32:
            data = np.ascontiguousarray(data, np.float32)
        else:
            data = np.ascontiguousarray(data, np.uint8)
            sq8_min = np.ascontiguousarray(sq8_min, np.float32)
            sq8_scale = np.ascontiguousarray(sq8_scale, np.float32)
        n, dim = data.shape
        h = lib().diskann_hip_register_db(data.ctypes.data_as(C.c_void_p), n, dim, fmt, _ptr(sq8_min, C.c_float),
                                          _ptr(sq8_scale, C.c_float))
        if not h:
            raise HipAnnError("diskann_hip_register_db failed")
        self._h = C.c_void_p(h)
        self.n, self.dim, self.fmt = n, dim, fmt

    def close(self):
        if getattr(self, "_h", None):
            lib().diskann_hip_release_db(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def distances_ids(self, queries, ids, query_map, metric: int = METRIC_L2) -> np.ndarray:
        q = np.ascontiguousarray(queries, np.float32)
        ids = np.ascontiguousarray(ids, np.uint32)
        qm = np.ascontiguousarray(query_map, np.uint32)
        out = np.empty(ids.size, np.float32)
        rc = lib().diskann_hip_multi_batch_distances_ids(self._h, _ptr(q, C.c_float), q.shape[0],
                                                         _ptr(ids, C.c_uint32), _ptr(qm, C.c_uint32), ids.size,
                                                         metric, _ptr(out, C.c_float))
        if rc != 0:
            raise HipAnnError("diskann_hip_multi_batch_distances_ids failed")
        return out

    def set_kernel_timing(self, on: bool) -> None:
        """Record HIP events around every id-gather launch from now on (resets the record)."""
        if lib().diskann_hip_set_kernel_timing(self._h, 1 if on else 0) != 0:
            raise HipAnnError("diskann_hip_set_kernel_timing failed")

    def kernel_stats(self) -> Tuple[float, int]:
        """(summed kernel ms, launches) since set_kernel_timing(True)."""
        ms, n = C.c_double(0.0), C.c_int64(0)
        if lib().diskann_hip_kernel_stats(self._h, C.byref(ms), C.byref(n)) != 0:
            raise HipAnnError("diskann_hip_kernel_stats failed")
        return ms.value, n.value

    def register_graph(self, adjacency: np.ndarray) -> None:
        """Upload the n x R adjacency (u32::MAX padding) for search_batch_resident."""
        adj = np.ascontiguousarray(adjacency, np.uint32)
        if adj.ndim != 2 or adj.shape[0] != self.n:
            raise HipAnnError("adjacency must be (n, R)")
        if lib().diskann_hip_register_graph(self._h, _ptr(adj, C.c_uint32), adj.shape[1]) != 0:
            raise HipAnnError("diskann_hip_register_graph failed")

    def search_batch_resident(self, entry_points, queries, k: int, l_search: int, metric: int = METRIC_L2):
        """DiskProvider::search_batch with the traversal itself on the GPU (one 2-wavefront workgroup per query).
        Returns (ids, dists, stats)."""
        eps = np.ascontiguousarray(entry_points, np.uint32)
        q = np.ascontiguousarray(queries, np.float32)
        nq = q.shape[0]
        kk = min(k, self.n)
        out_i = np.empty((nq, kk), np.int64)
        out_d = np.empty((nq, kk), np.float32)
        stats = np.zeros(4, np.int64)
        eb = _err()
        rc = lib().diskann_hip_search_batch_resident(self._h, _ptr(eps, C.c_uint32), eps.size, _ptr(q, C.c_float),
                                                     nq, kk, l_search, metric, _ptr(out_i, C.c_int64),
                                                     _ptr(out_d, C.c_float), _ptr(stats, C.c_int64), eb, 1024)
        _check(rc, eb)
        return out_i, out_d, {"evals": int(stats[0]), "steps": int(stats[1]), "pops": int(stats[2]),
                              "host_requeries": int(stats[3])}

    def search_batch_resident_device(self, entry_points, nq: int, q_ptr: int, k: int, l_search: int, i_ptr: int,
                                     d_ptr: int, metric: int = METRIC_L2, stream: int = 0):
        """Device-pointer form (queries nq x dim fp32, outputs nq x k int64 / fp32 in HBM)."""
        eps = np.ascontiguousarray(entry_points, np.uint32)
        stats = np.zeros(4, np.int64)
        eb = _err()
        rc = lib().diskann_hip_search_batch_resident_device(self._h, _ptr(eps, C.c_uint32), eps.size,
                                                            C.c_void_p(q_ptr), nq, k, l_search, metric,
                                                            C.c_void_p(i_ptr), C.c_void_p(d_ptr),
                                                            _ptr(stats, C.c_int64), C.c_void_p(stream or None), eb,
                                                            1024)
        _check(rc, eb)
        return {"evals": int(stats[0]), "steps": int(stats[1]), "pops": int(stats[2]),
                "host_requeries": int(stats[3])}

    def search_batch(self, adjacency: np.ndarray, entry_points, queries, k: int, l_search: int,
                     metric: int = METRIC_L2):
        """DiskProvider::search_batch (disk_provider.rs:470-652) with every BFS step's distances computed
        on the GPU from this HBM-resident DB (native C++ BFS in libhipann).  Returns (ids, dists, stats)."""
        adj = np.ascontiguousarray(adjacency, np.uint32)
        eps = np.ascontiguousarray(entry_points, np.uint32)
        q = np.ascontiguousarray(queries, np.float32)
        nq = q.shape[0]
        kk = min(k, self.n)
        out_i = np.empty((nq, kk), np.int64)
        out_d = np.empty((nq, kk), np.float32)
        stats = np.zeros(4, np.int64)
        eb = _err()
        rc = lib().diskann_hip_search_batch(self._h, _ptr(adj, C.c_uint32), adj.shape[1], _ptr(eps, C.c_uint32),
                                            eps.size, _ptr(q, C.c_float), nq, kk, l_search, metric,
                                            _ptr(out_i, C.c_int64), _ptr(out_d, C.c_float), _ptr(stats, C.c_int64),
                                            eb, 1024)
        _check(rc, eb)
        return out_i, out_d, {"evals": int(stats[0]), "steps": int(stats[1]), "gpu_calls": int(stats[2])}
