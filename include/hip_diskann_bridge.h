/*
 * hip_diskann_bridge.h — C ABI for DiskANN batch distances on MI355X.
 *
 * Signature-identical replacement of the reference's Metal bridge
 * (src/include/metal_diskann_bridge.h:8-23, implemented in src/metal_diskann_bridge.mm:155-323,
 * stubbed in src/metal_diskann_stub.cpp:9-24).  Callers in the reference:
 *   - rust_lib/src/metal_ffi.rs:10-30 (→ DiskProvider::search / search_batch,
 *     rust_lib/src/disk_provider.rs:417-445, :590-627; Provider::search_batch, provider.rs:385-415)
 *   - src/ann_search.cpp:723-732 (vector_distances → ComputeDistances)
 *
 * Semantics (diskann_distance.metal:15-194, rust_lib/src/distance.rs:15-24):
 *   metric 0 = L2  → out[i] = Σ_j (q_j − c_j)²           (squared Euclidean)
 *   metric 1 = IP  → out[i] = −Σ_j q_j · c_j             (negated dot; lower = more similar)
 * Returns 0 on success, −1 on invalid arguments (n/total_n/nq/dim ≤ 0, NULL pointers, a metric
 * other than 0/1, a query_map entry ≥ nq) or device failure; the caller then computes on the CPU
 * (disk_provider.rs:436-453, provider.rs:407-426).  Calls are synchronous; the caller owns all
 * buffers and nothing is retained after return.  Unlike the Metal bridge (non-atomic ring index,
 * metal_diskann_bridge.mm:52-53, :119-120) every entry point is thread-safe: each calling thread
 * gets its own stream and staging buffers.
 *
 * For drop-in linking the library also exports the reference's own `diskann_metal_*` names
 * (aliases of the `diskann_hip_*` functions), so rust_lib's metal_ffi.rs links unchanged.
 *
 * Extension: an HBM-resident database and an id-based call, so a
 * lock-step BFS step ships only candidate ids (4 B) instead of candidate vectors (4·dim B).
 * fmt 0 = fp32 rows (n*dim floats); fmt 1 = SQ8 codes (n*dim uint8) with per-dimension `sq8_min`
 * and `sq8_scale` (dequant v = (q/255)·scale + min, rust_lib/src/provider.rs:140-146, :161-210).
 */
#ifndef HIP_DISKANN_BRIDGE_H
#define HIP_DISKANN_BRIDGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Returns 1 if HIP DiskANN acceleration is available, 0 otherwise (metal_diskann_bridge.h:8). */
int diskann_hip_available(void);

/* One query (dim floats) vs n contiguous candidates (n*dim floats) → out_distances[n]
 * (metal_diskann_bridge.h:10-15). */
int diskann_hip_batch_distances(const float *query, const float *candidates, int n, int dim, int metric,
                                float *out_distances);

/* nq queries (nq*dim), total_n candidates (total_n*dim); candidate i is compared with
 * queries[query_map[i]] (metal_diskann_bridge.h:17-23). */
int diskann_hip_multi_batch_distances(const float *queries, const float *candidates, const unsigned int *query_map,
                                      int total_n, int nq, int dim, int metric, float *out_distances);

/* Drop-in aliases of the reference names (same semantics as the diskann_hip_* functions). */
int diskann_metal_available(void);
int diskann_metal_batch_distances(const float *query, const float *candidates, int n, int dim, int metric,
                                  float *out_distances);
int diskann_metal_multi_batch_distances(const float *queries, const float *candidates, const unsigned int *query_map,
                                        int total_n, int nq, int dim, int metric, float *out_distances);

/* ---- extension: HBM-resident database + id gather ---------------------------------------- */

#define DISKANN_HIP_FMT_F32 0
#define DISKANN_HIP_FMT_SQ8 1

/* Upload n vectors (fmt as above) to HBM on the current device; returns a handle or NULL. */
void *diskann_hip_register_db(const void *data, int64_t n, int dim, int fmt, const float *sq8_min,
                              const float *sq8_scale);

/* out[i] = dist(queries[query_map[i]], db[ids[i]]) for i < total_n.  ids ≥ n are an error (−1).
 * Host pointers; synchronous. */
int diskann_hip_multi_batch_distances_ids(void *db, const float *queries, int nq, const unsigned int *ids,
                                          const unsigned int *query_map, int total_n, int metric,
                                          float *out_distances);

/* Same with every buffer already in HBM (asynchronous on `stream`, a hipStream_t; NULL = the
 * default/null stream).  For benchmarking the kernel with resident inputs. */
int diskann_hip_multi_batch_distances_ids_device(void *db, const float *queries_dev, int nq,
                                                 const unsigned int *ids_dev, const unsigned int *query_map_dev,
                                                 int total_n, int metric, float *out_dev, void *stream);

/* Lock-step multi-query best-first search over the registered DB — DiskProvider::search_batch
 * (rust_lib/src/disk_provider.rs:470-652: pop the best candidate per active query, stop when
 * |result| >= L and it is worse than result[L-1], expand unvisited neighbours, insert_result
 * :656-678) with every step's distances computed by the id-gather kernel.  adjacency: n*R uint32,
 * padded with UINT32_MAX (rust_lib/src/file_format.rs:3-18).  Outputs nq*k labels (−1 past the
 * result) and distances (FLT_MAX past the result).  stats (may be NULL): [0] distance evaluations,
 * [1] lock-step iterations, [2] GPU calls, [3] reserved.  Returns 0 / −1 (message in err_buf). */
int diskann_hip_search_batch(void *db, const uint32_t *adjacency, int R, const uint32_t *entry_points, int n_ep,
                             const float *queries, int nq, int k, int l_search, int metric, int64_t *out_ids,
                             float *out_dists, int64_t *stats, char *err_buf, int err_len);

/* ---- extension: GPU-resident traversal ---------------------------------------------------------
 * The whole DiskProvider::search_batch (disk_provider.rs:470-678) on the device: one wavefront per
 * query runs the reference's state machine (sorted result list of L, pop of the smallest unexpanded
 * (dist, id), neighbour expansion up to the first u32::MAX, visited set, insert_result with Rust's
 * binary_search_by) against the HBM-resident DB and adjacency — no per-step host round trip.
 * Results equal diskann_hip_search_batch's up to fp32 summation order.  Shapes the kernel does not
 * cover (R > 64, n_ep > 64, L > 256, d beyond 2048 SQ8 / 2048 fp32 or not a multiple of 16 / 4) and
 * the rare query whose boundary-tie spill list overflows run through the host BFS transparently.
 * stats (may be NULL): [0] distance evaluations, [1] max BFS steps over queries (the lock-step count),
 * [2] node expansions (pops) on the GPU, [3] queries re-run on the host. */

/* Upload the graph (n x R uint32 adjacency, padded with UINT32_MAX) next to the registered DB. */
int diskann_hip_register_graph(void *db, const uint32_t *adjacency, int R);

/* Host pointers; synchronous. */
int diskann_hip_search_batch_resident(void *db, const uint32_t *entry_points, int n_ep, const float *queries, int nq,
                                      int k, int l_search, int metric, int64_t *out_ids, float *out_dists,
                                      int64_t *stats, char *err_buf, int err_len);

/* queries / out_ids / out_dists in HBM; launched on `stream` (hipStream_t, NULL = the DB's stream); returns
 * after the traversal finished (it reads back the per-query flags). */
int diskann_hip_search_batch_resident_device(void *db, const uint32_t *entry_points, int n_ep,
                                             const float *queries_dev, int nq, int k, int l_search, int metric,
                                             int64_t *out_ids_dev, float *out_dists_dev, int64_t *stats, void *stream,
                                             char *err_buf, int err_len);

int64_t diskann_hip_db_size(void *db);

/* Measurement: record HIP events around every id-gather kernel launch of `db` (on its stream) from now
 * on (on != 0; resets the record), and read back the summed kernel time and the launch count. */
int diskann_hip_set_kernel_timing(void *db, int on);
int diskann_hip_kernel_stats(void *db, double *total_ms, int64_t *launches);
void diskann_hip_release_db(void *db);

#ifdef __cplusplus
}
#endif

#endif /* HIP_DISKANN_BRIDGE_H */
