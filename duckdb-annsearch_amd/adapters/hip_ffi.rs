//! FFI bridge to MI355X batch distance computation — drop-in replacement of
//! rust_lib/src/metal_ffi.rs.  The callers name the module by full path
//! (`crate::metal_ffi::MIN_GPU_WORK`, `crate::metal_ffi::metal_batch_distances`,
//! `crate::metal_ffi::metal_multi_batch_distances`: disk_provider.rs:417, :427, :590, :601;
//! provider.rs:385, :396), so the swap is one line in rust_lib/src/lib.rs:6:
//!
//!     #[path = "hip_ffi.rs"] pub mod metal_ffi;
//!
//! and this module exports the reference names (`is_metal_available`, `metal_batch_distances`,
//! `metal_multi_batch_distances`, `MIN_GPU_WORK`, `MIN_GPU_WORK_ONESHOT`) next to the `hip_*` ones.
//! (Alternatively keep metal_ffi.rs unchanged and link libhipann.so, which also exports the
//! `diskann_metal_*` C names.)
//!
//! The implementation lives in libhipann.so (duckdb-annsearch_amd/csrc/diskann.hip); its C ABI is
//! include/hip_diskann_bridge.h.  Symbols are resolved at link time when the Rust static lib is
//! linked with the C++ extension (metal_ffi.rs:5-6, CMakeLists.txt:231-236).
//!
//! Source only in this repository (no cargo/rustc in the build image); INTEGRATION.md shows the
//! Cargo / CMake wiring.

use std::sync::atomic::{AtomicI32, Ordering};

extern "C" {
    fn diskann_hip_available() -> i32;
    fn diskann_hip_batch_distances(
        query: *const f32,
        candidates: *const f32,
        n: i32,
        dim: i32,
        metric: i32,
        out_distances: *mut f32,
    ) -> i32;
    fn diskann_hip_multi_batch_distances(
        queries: *const f32,
        candidates: *const f32,
        query_map: *const u32,
        total_n: i32,
        nq: i32,
        dim: i32,
        metric: i32,
        out_distances: *mut f32,
    ) -> i32;
    fn diskann_hip_register_db(
        data: *const core::ffi::c_void,
        n: i64,
        dim: i32,
        fmt: i32,
        sq8_min: *const f32,
        sq8_scale: *const f32,
    ) -> *mut core::ffi::c_void;
    fn diskann_hip_multi_batch_distances_ids(
        db: *mut core::ffi::c_void,
        queries: *const f32,
        nq: i32,
        ids: *const u32,
        query_map: *const u32,
        total_n: i32,
        metric: i32,
        out_distances: *mut f32,
    ) -> i32;
    fn diskann_hip_release_db(db: *mut core::ffi::c_void);
    fn diskann_hip_register_graph(db: *mut core::ffi::c_void, adjacency: *const u32, r: i32) -> i32;
    fn diskann_hip_search_batch_resident(
        db: *mut core::ffi::c_void,
        entry_points: *const u32,
        n_ep: i32,
        queries: *const f32,
        nq: i32,
        k: i32,
        l_search: i32,
        metric: i32,
        out_ids: *mut i64,
        out_dists: *mut f32,
        stats: *mut i64,
        err_buf: *mut core::ffi::c_char,
        err_len: i32,
    ) -> i32;
    fn diskann_hip_search_batch(
        db: *mut core::ffi::c_void,
        adjacency: *const u32,
        r: i32,
        entry_points: *const u32,
        n_ep: i32,
        queries: *const f32,
        nq: i32,
        k: i32,
        l_search: i32,
        metric: i32,
        out_ids: *mut i64,
        out_dists: *mut f32,
        stats: *mut i64,
        err_buf: *mut core::ffi::c_char,
        err_len: i32,
    ) -> i32;
}

/// Cached availability: -1 = unchecked, 0 = unavailable, 1 = available (metal_ffi.rs:33-34).
static HIP_STATUS: AtomicI32 = AtomicI32::new(-1);

/// Minimum n*dim to dispatch the reference-ABI (host candidate copy) path, measured on MI355X
/// (bench.py `reference_readme_batch_distances`, d = 768 sweep, profiles/r02/): the host-pointer call
/// costs ~21 us + ~0.15 us per 1000 floats (zero-copy from pinned staging up to 1 MiB), against a
/// 16-accumulator AVX2 CPU loop (the timing model of diskann-vector's SIMD distances this caller
/// falls back to) — break-even between n*d = 524K (GPU 103 us, CPU 90) and 1.05M (151 vs 176).
pub const MIN_GPU_WORK: usize = 786432;

/// One-shot threshold for vector_distances() (ann_search.cpp:699): its CPU side is the scalar
/// ComputeDistancesCPU loop, break-even measured at n*d = 65K (GPU 26.7 us, CPU 28.5).
pub const MIN_GPU_WORK_ONESHOT: usize = 65536;

/// Reference names (metal_ffi.rs:49, :67, :107): with `#[path = "hip_ffi.rs"] pub mod metal_ffi;` the
/// callers in disk_provider.rs / provider.rs resolve unchanged.
pub use self::hip_batch_distances as metal_batch_distances;
pub use self::hip_multi_batch_distances as metal_multi_batch_distances;
pub use self::is_hip_available as is_metal_available;

pub fn is_hip_available() -> bool {
    let status = HIP_STATUS.load(Ordering::Relaxed);
    if status >= 0 {
        return status == 1;
    }
    let avail = unsafe { diskann_hip_available() };
    HIP_STATUS.store(avail, Ordering::Relaxed);
    avail == 1
}

/// Same contract as metal_ffi::metal_batch_distances (metal_ffi.rs:67-95).
pub fn hip_batch_distances(query: &[f32], candidates: &[f32], n: usize, dim: usize, metric: u8, out: &mut [f32]) -> bool {
    if n == 0 || dim == 0 {
        return true;
    }
    if n * dim < MIN_GPU_WORK || !is_hip_available() {
        return false;
    }
    debug_assert_eq!(candidates.len(), n * dim);
    debug_assert!(out.len() >= n);
    let ret = unsafe {
        diskann_hip_batch_distances(query.as_ptr(), candidates.as_ptr(), n as i32, dim as i32, metric as i32, out.as_mut_ptr())
    };
    ret == 0
}

/// Same contract as metal_ffi::metal_multi_batch_distances (metal_ffi.rs:107-141).
pub fn hip_multi_batch_distances(
    queries: &[f32],
    candidates: &[f32],
    query_map: &[u32],
    total_n: usize,
    nq: usize,
    dim: usize,
    metric: u8,
    out: &mut [f32],
) -> bool {
    if total_n == 0 || nq == 0 || dim == 0 {
        return true;
    }
    if !is_hip_available() {
        return false;
    }
    debug_assert_eq!(queries.len(), nq * dim);
    debug_assert_eq!(candidates.len(), total_n * dim);
    debug_assert_eq!(query_map.len(), total_n);
    let ret = unsafe {
        diskann_hip_multi_batch_distances(
            queries.as_ptr(),
            candidates.as_ptr(),
            query_map.as_ptr(),
            total_n as i32,
            nq as i32,
            dim as i32,
            metric as i32,
            out.as_mut_ptr(),
        )
    };
    ret == 0
}

/// HBM-resident database for DiskProvider: register once at
/// DiskProvider::open, then each lock-step BFS step ships only (id, query) pairs.
pub struct HipDiskDb {
    h: *mut core::ffi::c_void,
    n: usize,
    dim: usize,
}

unsafe impl Send for HipDiskDb {}
unsafe impl Sync for HipDiskDb {}

impl HipDiskDb {
    /// fp32 rows (the .diskann vector segment, e.g. straight from the mmap).
    pub fn from_f32(vectors: &[f32], n: usize, dim: usize) -> Option<Self> {
        // the C side copies n × dim values: a shorter slice would be read out of bounds
        if !is_hip_available() || dim == 0 || dim > i32::MAX as usize || vectors.len() < n.checked_mul(dim)? {
            return None;
        }
        let h = unsafe {
            diskann_hip_register_db(vectors.as_ptr() as *const _, n as i64, dim as i32, 0, std::ptr::null(), std::ptr::null())
        };
        if h.is_null() { None } else { Some(HipDiskDb { h, n, dim }) }
    }

    /// SQ8 codes with the provider's per-dimension min / scale (provider.rs:25-38).
    pub fn from_sq8(codes: &[u8], n: usize, dim: usize, min: &[f32], scale: &[f32]) -> Option<Self> {
        if !is_hip_available()
            || dim == 0
            || dim > i32::MAX as usize
            || codes.len() < n.checked_mul(dim)?
            || min.len() < dim
            || scale.len() < dim
        {
            return None;
        }
        let h = unsafe {
            diskann_hip_register_db(codes.as_ptr() as *const _, n as i64, dim as i32, 1, min.as_ptr(), scale.as_ptr())
        };
        if h.is_null() { None } else { Some(HipDiskDb { h, n, dim }) }
    }

    /// Slice shapes of a query batch: nq × dim queries, every count within the C ABI's i32.
    fn batch_ok(&self, queries: &[f32], nq: usize, k: usize) -> bool {
        nq <= i32::MAX as usize
            && k <= i32::MAX as usize
            && nq.checked_mul(self.dim).map_or(false, |m| queries.len() >= m)
    }

    /// out[i] = dist(queries[query_map[i]], db[ids[i]]) — replaces the gather + metal_multi_batch_distances
    /// pair of disk_provider.rs:592-610.  false ⇒ caller computes on the CPU.
    pub fn multi_batch_distances_ids(&self, queries: &[f32], nq: usize, ids: &[u32], query_map: &[u32], metric: u8, out: &mut [f32]) -> bool {
        if ids.is_empty() {
            return true;
        }
        // every index the kernel follows must be inside the slices it reads (ids < n, query_map < nq)
        if !self.batch_ok(queries, nq, 0)
            || ids.len() > i32::MAX as usize
            || query_map.len() != ids.len()
            || out.len() < ids.len()
            || ids.iter().any(|&i| i as usize >= self.n)
            || query_map.iter().any(|&q| q as usize >= nq)
        {
            return false;
        }
        let ret = unsafe {
            diskann_hip_multi_batch_distances_ids(
                self.h,
                queries.as_ptr(),
                nq as i32,
                ids.as_ptr(),
                query_map.as_ptr(),
                ids.len() as i32,
                metric as i32,
                out.as_mut_ptr(),
            )
        };
        ret == 0
    }
}

/// (nq × k) C-ABI outputs → DiskProvider::search_batch's return shape: per query the first k
/// (id, dist) pairs, stopping at the first −1 label (the slots past a short result, ffi.rs:759-762).
fn collect_results(ids: &[i64], dists: &[f32], nq: usize, k: usize) -> Vec<Vec<(u64, f32)>> {
    (0..nq)
        .map(|q| {
            ids[q * k..(q + 1) * k]
                .iter()
                .zip(&dists[q * k..(q + 1) * k])
                .take_while(|(id, _)| **id >= 0)
                .map(|(id, d)| (*id as u64, *d))
                .collect()
        })
        .collect()
}

impl HipDiskDb {
    /// Upload the graph (the .diskann adjacency segment: n × R u32, u32::MAX padding, file_format.rs:3-18)
    /// next to the registered vectors, once at DiskProvider::open.  After this, search_batch_resident runs
    /// the whole lock-step BFS of DiskProvider::search_batch (disk_provider.rs:470-652) on the GPU.
    pub fn register_graph(&self, adjacency: &[u32], max_degree: usize) -> bool {
        // the C side copies n × max_degree ids (diskann.hip diskann_hip_register_graph)
        if max_degree == 0 || max_degree > i32::MAX as usize || self.n.checked_mul(max_degree) != Some(adjacency.len()) {
            return false;
        }
        unsafe { diskann_hip_register_graph(self.h, adjacency.as_ptr(), max_degree as i32) == 0 }
    }

    /// DiskProvider::search_batch with the traversal on the GPU (one workgroup per query runs the reference's
    /// state machine: pop / stop rule / visited set / insert_result, disk_provider.rs:539-678).  `queries_flat`
    /// is nq × dim.  None ⇒ the caller runs its own lock-step loop (host BFS + id-gather, or the CPU).
    pub fn search_batch_resident(
        &self,
        entry_points: &[u32],
        queries_flat: &[f32],
        nq: usize,
        k: usize,
        l_search: usize,
        metric: u8,
    ) -> Option<Vec<Vec<(u64, f32)>>> {
        if nq == 0 || k == 0 {
            return Some(vec![Vec::new(); nq]);
        }
        if !self.batch_ok(queries_flat, nq, k) || l_search > i32::MAX as usize || entry_points.len() > i32::MAX as usize {
            return None;
        }
        let mut ids = vec![-1i64; nq * k];
        let mut dists = vec![f32::MAX; nq * k];
        let mut stats = [0i64; 4];
        let mut err = [0 as core::ffi::c_char; 256];
        let ret = unsafe {
            diskann_hip_search_batch_resident(
                self.h,
                entry_points.as_ptr(),
                entry_points.len() as i32,
                queries_flat.as_ptr(),
                nq as i32,
                k as i32,
                l_search as i32,
                metric as i32,
                ids.as_mut_ptr(),
                dists.as_mut_ptr(),
                stats.as_mut_ptr(),
                err.as_mut_ptr(),
                err.len() as i32,
            )
        };
        if ret != 0 {
            return None;
        }
        Some(collect_results(&ids, &dists, nq, k))
    }

    /// The same search with the BFS on the host (native C++ lock-step loop in libhipann) and every step's
    /// distances from the id-gather kernel over this HBM-resident DB — the reference's structure with the
    /// candidate copy replaced by ids.  Used when the graph was not registered.
    pub fn search_batch_host_bfs(
        &self,
        adjacency: &[u32],
        max_degree: usize,
        entry_points: &[u32],
        queries_flat: &[f32],
        nq: usize,
        k: usize,
        l_search: usize,
        metric: u8,
    ) -> Option<Vec<Vec<(u64, f32)>>> {
        if nq == 0 || k == 0 {
            return Some(vec![Vec::new(); nq]);
        }
        if !self.batch_ok(queries_flat, nq, k)
            || l_search > i32::MAX as usize
            || entry_points.len() > i32::MAX as usize
            || max_degree == 0
            || max_degree > i32::MAX as usize
            || self.n.checked_mul(max_degree) != Some(adjacency.len())
        {
            return None;
        }
        let mut ids = vec![-1i64; nq * k];
        let mut dists = vec![f32::MAX; nq * k];
        let mut stats = [0i64; 4];
        let mut err = [0 as core::ffi::c_char; 256];
        let ret = unsafe {
            diskann_hip_search_batch(
                self.h,
                adjacency.as_ptr(),
                max_degree as i32,
                entry_points.as_ptr(),
                entry_points.len() as i32,
                queries_flat.as_ptr(),
                nq as i32,
                k as i32,
                l_search as i32,
                metric as i32,
                ids.as_mut_ptr(),
                dists.as_mut_ptr(),
                stats.as_mut_ptr(),
                err.as_mut_ptr(),
                err.len() as i32,
            )
        };
        if ret != 0 {
            return None;
        }
        Some(collect_results(&ids, &dists, nq, k))
    }
}

impl Drop for HipDiskDb {
    fn drop(&mut self) {
        unsafe { diskann_hip_release_db(self.h) }
    }
}
