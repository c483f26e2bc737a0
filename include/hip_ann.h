/*
 * hip_ann.h — C ABI of the MI355X search backend for the DuckDB `ann` extension's FAISS indexes.
 *
 * This is the plain-C layer that sits UNDER the extension's `GpuBackend` interface
 * (reference: src/include/gpu_backend.hpp:12-33).  The reference implements that interface with
 * faiss-metal (`MetalGpuBackend::CpuToGpu`, src/gpu_backend_metal.mm:42-60), which deep-copies a
 * FAISS `IndexFlat` / `IndexIVFFlat` into a `faiss::Index` subclass whose `search()` runs on the GPU
 * (faiss-metal/src/MetalIndexFlat.mm:294-369, faiss-metal/src/MetalIndexIVFFlat.mm:122-256).
 * Here the GPU index is an opaque handle behind these entry points; the C++ adapter
 * `duckdb-annsearch_amd/adapters/gpu_backend_hip.cpp` wraps them into `faiss::Index` subclasses.
 *
 * Conventions (mirroring the extension's Rust FFI, rust_lib/src/ffi.rs:14-23):
 *   - every fallible call takes `char *err_buf, int err_len`; on failure it writes a NUL-terminated
 *     message there (when err_buf != NULL) and returns -1 (int) or NULL (handle);
 *   - the caller owns every host buffer; the library copies at create time and writes the outputs
 *     synchronously before returning (host-pointer API);
 *   - handles are opaque; hipann_free(NULL) is a no-op; a handle serialises its own calls with a
 *     mutex (one HIP stream + scratch arena per handle), so concurrent DuckDB connections are safe;
 *   - metric: 0 = L2 (squared Euclidean, ascending), 1 = inner product (raw dot, descending) —
 *     faiss::MetricType values METRIC_INNER_PRODUCT=0 / METRIC_L2=1 are NOT used here; see HIPANN_*;
 *   - search outputs follow MetalIndexFlat::search (MetalIndexFlat.mm:294-369): D is nq*k floats,
 *     I is nq*k int64 labels; slots beyond min(k, ntotal) hold (+inf | -inf, -1); k <= 0 is an error;
 *     equal distances are ordered by ascending label (FAISS heap id tie-break).
 *
 * There is no CPU implementation behind this ABI: without a HIP device every compute entry point
 * fails with -1 ("no HIP device").  The CPU path is the extension's own FAISS CPU index.
 */
#ifndef HIP_ANN_H
#define HIP_ANN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIPANN_METRIC_L2 0
#define HIPANN_METRIC_IP 1

/* Largest k the GPU path serves (faiss-metal's block select tops out at 2048, MetalSelect.mm:53-57). */
#define HIPANN_MAX_K 2048
/* EnsureGpuIndex's AUTO gate on MI355X (replaces ntotal >= 256 && d >= 128, faiss_index.cpp:128-143): upload
 * when ntotal * d >= HIPANN_AUTO_MIN_WORK.  Measured (bench.py flat_auto_gate): the host-pointer nq = 1 call
 * (the extension's per-query search, faiss_index.cpp:737) beats the CPU path's per-query scan from
 * ntotal * d ~ 0.6-1.5M floats at d = 128 and 768. */
#define HIPANN_AUTO_MIN_WORK 1048576

/* 1 when at least one gfx950 HIP device is usable, else 0.  Replaces
 * MetalGpuBackend::IsAvailable (gpu_backend_metal.mm:20-31, :33-35). */
int hipann_available(void);

/* Number of visible HIP devices (0 without a GPU). */
int hipann_device_count(void);

/* Human-readable device description, e.g. "AMD Instinct MI355X (gfx950, 256 CUs, 288 GB) x8".
 * Replaces MetalGpuBackend::DeviceInfo (gpu_backend_metal.mm:37-43) → faiss_gpu_info().device
 * (src/faiss_fn_gpu.cpp:42-45).  Returns the string length, or -1. */
int hipann_device_info(char *buf, int buf_len);

/* Peer access of a (multi-device) Flat or IVF handle, set when it was created: hipann_flat_create /
 * hipann_ivf_create with devices[] call hipDeviceCanAccessPeer both ways between every shard's device and the first
 * shard's, then hipDeviceEnablePeerAccess, so the per-shard top-k gather (hipMemcpyPeerAsync onto the first device)
 * rides xGMI.  state[s] (cap >= shard count; NULL to ask the count): 2 = on the first shard's device (no peer copy),
 * 1 = peer access enabled both ways, 0 = not available (the runtime stages the copy through host memory).  Returns the
 * shard count, or -1. */
int hipann_peer_access(void *index, int *state, int cap, char *err_buf, int err_len);

/* ---------------------------------------------------------------------------------------------
 * Flat (brute force) — replaces index_cpu_to_metal + MetalIndexFlat (MetalIndexFlat.mm:504-515,
 * :173-292 add, :294-369 search).
 * ------------------------------------------------------------------------------------------- */

/* Create a Flat index over n row-major fp32 vectors `xb` (n*d floats, host memory).  Rows are
 * sharded contiguously over `devices[0..ndev)` (NULL/0 = device 0); labels are 0..n-1. */
void *hipann_flat_create(int d, int metric, const float *xb, int64_t n, const int *devices, int ndev,
                         char *err_buf, int err_len);

/* Append n more vectors (labels continue from ntotal) — MetalIndexFlat::add (MetalIndexFlat.mm:173-292). */
int hipann_flat_add(void *index, const float *xb, int64_t n, char *err_buf, int err_len);

/* Search nq queries `xq` (nq*d floats, host).  D: nq*k floats, I: nq*k int64 (host). */
int hipann_flat_search(void *index, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I,
                       char *err_buf, int err_len);

/* Copy vector `key` back to host (faiss::Index::reconstruct; MetalIndexFlat::reconstruct). */
int hipann_flat_reconstruct(void *index, int64_t key, float *out, char *err_buf, int err_len);

/* Copy rows [i0, i0+n) back to host (faiss::Index::reconstruct_n; GpuToCpu of a Flat index,
 * gpu_backend_metal.mm:68-72 → index_metal_to_cpu). */
int hipann_flat_reconstruct_n(void *index, int64_t i0, int64_t n, float *out, char *err_buf, int err_len);

/* q·x form of the batched (nq >= 20, FAISS's BLAS threshold) distance path, ‖q‖² + ‖x‖² − 2·q·x.
 * HIPANN_FLAT_FORM_FP32: exact fp32 products on the fp32 matrix cores (v_mfma_f32_32x32x2_f32).
 * HIPANN_FLAT_FORM_SPLIT3: both operands split into three round-to-nearest bf16 terms, the
 * six products above 2^-26 relative on the bf16 matrix cores, fp32 accumulation — fp32-level products
 * at several times the fp32 rate.  HIPANN_FLAT_FORM_SPLIT2: two terms, three products (≈2^-16
 * relative per product; measurement only).  HIPANN_FLAT_FORM_SPLIT2_EXACT: the SPLIT2 scan keeps the
 * 16 best rows (32 for IP) per database split and query only as a filter; every returned distance is
 * recomputed in FAISS's direct fp32 form (Σ(q−x)² / q·x) and a per-query bound (|scan key − exact| ≤
 * 2^-12·(‖q‖² + max‖x‖²)) proves no pruned row reaches the top-k — queries that fail it re-run on
 * SPLIT3 (k ≤ 12; larger k use SPLIT3).  HIPANN_FLAT_FORM_BF16_EXACT: the same filter +
 * rerank, the scan computing ONE bf16 product per element over a tiled bf16 image of the rows (built
 * once); the bound is the Cauchy-Schwarz bound of the measured bf16 residuals.  Returns 0, or -1 for a
 * bad handle / form. */
#define HIPANN_FLAT_FORM_FP32 0
#define HIPANN_FLAT_FORM_SPLIT3 1
#define HIPANN_FLAT_FORM_SPLIT2 2
#define HIPANN_FLAT_FORM_SPLIT2_EXACT 3
#define HIPANN_FLAT_FORM_BF16_EXACT 4
/* HIPANN_FLAT_FORM_I8_EXACT (default): the BF16_EXACT pipeline with the scan over a tiled int8 image (per-row scale
 * max|x|/127, round to nearest) on the int8 matrix cores (v_mfma_i32_16x16x64_i8: exact int32 sums, twice the
 * bf16 rate, half its bytes per element) as the filter; a 64-deep filter, the bound from the measured int8
 * residuals of the rows and of each query.  Runs as the bounded passes only (>= 256 queries, >= 512K rows,
 * d <= 1024); elsewhere BF16_EXACT.  At 10M x 768, 1024 queries: 9.6 ms per batch against BF16_EXACT's 14.3,
 * identical ids. */
#define HIPANN_FLAT_FORM_I8_EXACT 5
int hipann_flat_set_form(void *index, int form);
int hipann_flat_get_form(void *index);
/* Queries re-run on HIPANN_FLAT_FORM_SPLIT3 since the index was created: those the exact forms' bound
 * check flagged and, for BF16_EXACT's bounded passes, the second rerank (every buffered candidate of
 * the query, certified against the pass bound) could not certify either; the exact results replace
 * the flagged ones. */
int64_t hipann_flat_rerank_fallbacks(void *index);
/* Host synchronisations made by the search calls of a Flat index since it was created.  hipann_flat_search
 * launches every shard (one per device of `devices[]`, each on its own stream) before it waits on any, gathers
 * and merges on the first device behind device-side event waits, and synchronises ONCE, which also reads every
 * shard's exact-form flag count; only a batch with flagged queries adds the syncs of their re-runs.  Building an
 * image after an add (first search) adds one.  -1 for a NULL / non-Flat handle. */
int64_t hipann_flat_host_syncs(void *index);

/* The path the last search of `index` (Flat or IVF) took: *form = the distance form its scan ran
 * (HIPANN_FLAT_FORM_* / HIPANN_IVF_FORM_*; the exact forms' re-runs of flagged queries not counted),
 * *filter_k = the exact forms' rerank depth (candidates per query; 0 = no rerank), *sublists = IVF sub-lists
 * per (query, list, chunk) slot (0 = one merged list).  Any output may be NULL.  Request_k above 12 — the
 * extension asks for k + |tombstones| (faiss_index.cpp:713-715) — stays on the exact forms up to 64 (Flat
 * bounded passes) / 60 (IVF) with a deeper filter; this is how tests and the bench see it.  Returns 0 / -1. */
int hipann_last_search_path(void *index, int *form, int *filter_k, int *sublists);

/* ---------------------------------------------------------------------------------------------
 * Device-resident variants (inputs and outputs already in HBM).  Used by the multi-GPU sharded
 * search (one process per GPU, partial top-k gathered over RCCL) and by bench.py, whose timed
 * region starts with the inputs resident.  `stream` is a hipStream_t (NULL = the default/null
 * stream, HIP's convention and PyTorch's default stream).  IVF: the call is asynchronous on that stream —
 * it returns with its kernels still queued (no host synchronisation, the exact forms' flagged queries
 * included: they are re-run on the device).  Flat: the exact forms (HIPANN_FLAT_FORM_SPLIT2_EXACT,
 * HIPANN_FLAT_FORM_BF16_EXACT, HIPANN_FLAT_FORM_I8_EXACT) synchronise the stream once per call to read the flagged-query count (twice
 * when the bounded passes' candidate rerank ran), and a table's first exact-form search also builds its bf16 /
 * int8 image and bound; the other forms return with their kernels queued.  Calls on one handle may use different streams
 * and execute in the order they were issued (the per-handle scratch is reused).  While every call comes on one stream
 * nothing is added between them (no event per call — an event marker costs ≈6 µs of idle GPU between back-to-back
 * searches).  The FIRST call on a different stream synchronises the handle's device once; from then on the handle
 * records an event at the end of every call and a call on another stream waits for it on the device
 * (hipStreamWaitEvent), so per-connection streams cost one marker per call, not a device-wide drain per alternation.
 * HIPANN_FENCE_EAGER=1 records the events from the first call.  The caller still orders its own buffers (queries
 * written / results read on other streams) with its own events.
 * Host waits (the Flat exact forms' flag count, host-pointer calls) poll for at most HIPANN_SPIN_US microseconds
 * (default 2000) and then block in hipStreamSynchronize / hipEventSynchronize: short calls avoid the interrupt
 * wake-up (tens of µs), long ones do not hold a host core for the whole kernel.  HIPANN_SPIN_WAIT=0: always block.
 * ------------------------------------------------------------------------------------------- */

/* Wrap (copy=0: borrow, caller keeps it alive) or copy (copy=1) an HBM matrix of n*d fp32 on
 * `device`.  Labels are label_offset + row. */
void *hipann_flat_create_device(int d, int metric, const float *xb_dev, int64_t n, int device, int copy,
                                int64_t label_offset, char *err_buf, int err_len);

int hipann_flat_search_device(void *index, int64_t nq, const float *xq_dev, int64_t k, float *D_dev,
                              int64_t *I_dev, void *stream, char *err_buf, int err_len);

/* k-way merge of `nparts` partial results laid out [part][nq][k] (device memory) into [nq][k]:
 * the k best by (distance, label) — ascending for L2, descending for IP; -1 labels are ignored.
 * The merge step after the RCCL allgather of per-GPU partial top-k. */
int hipann_merge_topk_device(int metric, int nparts, int64_t nq, int64_t k, const float *D_parts,
                             const int64_t *I_parts, float *D_out, int64_t *I_out, void *stream,
                             char *err_buf, int err_len);

/* The same merge over packed parts, the layout of ONE all-gather (sharded.py): part p sits at
 * parts + p*part_bytes and holds [labels int64 nq*k][distances fp32 nq*k] (part_bytes >= 12*nq*k, a
 * multiple of 8).  One collective moves each rank's distances and labels together. */
int hipann_merge_topk_packed_device(int metric, int nparts, int64_t nq, int64_t k, const void *parts,
                                    int64_t part_bytes, float *D_out, int64_t *I_out, void *stream,
                                    char *err_buf, int err_len);

/* ---------------------------------------------------------------------------------------------
 * IVFFlat — replaces index_cpu_to_metal_ivf + MetalIndexIVFFlat (MetalIndexIVFFlat.mm:283-326,
 * :122-256).  Lists are given in CSR form exactly as FAISS's ArrayInvertedLists hold them:
 * list l owns rows [list_offsets[l], list_offsets[l+1]) of `codes` (raw fp32 vectors — IVFFlat
 * stores unresidualised codes) and of `ids` (int64 labels).
 * ------------------------------------------------------------------------------------------- */

void *hipann_ivf_create(int d, int metric, int nlist, int nprobe, const float *centroids,
                        const int64_t *list_offsets, const int64_t *ids, const float *codes,
                        const int *devices, int ndev, char *err_buf, int err_len);

/* Device-resident IVF (single device): centroids (nlist*d), ids (n int64) and codes (n*d fp32)
 * already in HBM on `device`, list_offsets on the host.  copy=0 borrows the buffers. */
void *hipann_ivf_create_device(int d, int metric, int nlist, int nprobe, const float *centroids_dev,
                               const int64_t *list_offsets, const int64_t *ids_dev, const float *codes_dev,
                               int device, int copy, char *err_buf, int err_len);

int hipann_ivf_search(void *index, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I,
                      char *err_buf, int err_len);

/* Search with a per-call nprobe (SearchParametersIVF::nprobe, faiss_index.cpp:720-726); nprobe <= 0 uses
 * the index's.  The value is read under the handle's lock, so concurrent callers with different nprobe
 * never see each other's (the race of a set_nprobe + search pair). */
int hipann_ivf_search_np(void *index, int nprobe, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I,
                         char *err_buf, int err_len);

int hipann_ivf_search_device(void *index, int64_t nq, const float *xq_dev, int64_t k, float *D_dev,
                             int64_t *I_dev, void *stream, char *err_buf, int err_len);

/* Probe lists chosen by the last search (nq*nprobe int64, host) — for parity tests. */
int hipann_ivf_last_probes(void *index, int64_t *probes, int64_t cap, char *err_buf, int err_len);
/* The coarse step partitioned over ranks (list-sharded multi-GPU IVF): each rank computes the probe
 * lists of ITS slice of the batch (hipann_ivf_coarse_device: FAISS quantizer->search(nq, x, nprobe) on the
 * coarse quantizer, probes_dev = nq × min(nprobe, nlist) int64 list ids in probe order), one all-gather makes the
 * whole batch's lists, and hipann_ivf_search_probes_device searches every query with those probe lists instead of
 * running the coarse step again — bit-identical to the replicated scheme (a query's probe list does not depend on
 * the other queries of the batch while every slice has >= 20 queries, FAISS's BLAS-form threshold).  Both are
 * asynchronous on `stream`, like hipann_ivf_search_device; single-device handles only.  0 / -1. */
int hipann_ivf_coarse_device(void *index, int64_t nq, const float *xq_dev, int64_t *probes_dev, void *stream,
                             char *err_buf, int err_len);
int hipann_ivf_search_probes_device(void *index, int64_t nq, const float *xq_dev, const int64_t *probes_dev,
                                    int64_t k, float *D_dev, int64_t *I_dev, void *stream, char *err_buf, int err_len);

int hipann_ivf_set_nprobe(void *index, int nprobe);
int hipann_ivf_get_nprobe(void *index);
int hipann_ivf_nlist(void *index);

/* IndexIVFFlat::add_with_ids on the GPU copy (FAISS 1.13.2 IndexIVF::add_with_ids / add_core): the n rows
 * `xb` (host, n*d fp32) are assigned to their nearest centroid by the GPU coarse quantizer (k = 1, blocks
 * of 65536 rows as FAISS assigns them) and appended to their lists in insertion order, labels `ids`
 * (NULL: ntotal + i).  Replaces the reference's invalidate-on-append (faiss_index.cpp:469). */
int hipann_ivf_add(void *index, int64_t n, const float *xb, const int64_t *ids, char *err_buf, int err_len);

/* IVF training on the GPU — the k-means behind IndexIVFFlat::train (FAISS 1.13.2 IndexIVF::train_q1 →
 * Clustering::train), which the extension runs on the CPU at CREATE INDEX on a stride sample
 * (src/faiss_index.cpp:302-319).  From the n rows `x` (host, n*d fp32):
 *   1. training rows: when 0 < train_sample < n, rows (int64)(i * ((double)n / train_sample)), i < train_sample
 *      — the reference's deterministic stride sample (faiss_index.cpp:308-311); else all n rows (n must be >= nlist);
 *   2. at most 256 rows per centroid (FAISS's max_points_per_centroid): above that, a uniform subset;
 *   3. init: HIPANN_KMEANS_INIT_RANDOM (FAISS's: nlist random training rows) or HIPANN_KMEANS_INIT_PLUSPLUS
 *      (k-means++ D² sampling on the GPU);
 *   4. niter Lloyd iterations (FAISS's default 25): assignment by the GPU Flat search (k = 1, exact fp32
 *      products), centroids = fp64 means, FAISS's split of empty clusters, and for IP the spherical
 *      renormalisation (IndexIVF sets cp.spherical for METRIC_INNER_PRODUCT).
 * Every random draw comes from splitmix64(seed), so a result is reproducible and equals the oracle's
 * restatement (oracle/oracle.c oracle_kmeans_train) up to assignment ties; FAISS's own draws are not
 * reproduced.  centroids: nlist*d fp32 (host); list_sizes (optional, nlist int64): the cluster sizes of the
 * last iteration's assignment.  The result feeds hipann_ivf_create (or the CPU index's quantizer). */
#define HIPANN_KMEANS_INIT_RANDOM 0
#define HIPANN_KMEANS_INIT_PLUSPLUS 1
int hipann_ivf_train(int d, int metric, int nlist, int64_t n, const float *x, int64_t train_sample, int niter,
                     uint64_t seed, int init, int device, float *centroids, int64_t *list_sizes, char *err_buf,
                     int err_len);

/* The same with the rows and the result in HBM on `device` (x_dev: n*d fp32, centroids_dev: nlist*d fp32);
 * runs on `stream` and returns when the centroids are written. */
int hipann_ivf_train_device(int d, int metric, int nlist, int64_t n, const float *x_dev, int64_t train_sample,
                            int niter, uint64_t seed, int init, int device, float *centroids_dev, void *stream,
                            char *err_buf, int err_len);

/* Copy the index back to host in FAISS's ArrayInvertedLists CSR form — the inverse of hipann_ivf_create
 * (GpuBackend::GpuToCpu, gpu_backend_metal.mm:62-67 → index_metal_to_cpu_ivf, MetalIndexIVFFlat.mm:328-356):
 * centroids (nlist*d), list_offsets (nlist+1), ids (ntotal) and codes (ntotal*d, raw fp32 rows), lists in
 * order, rows in list order.  Any output may be NULL (skipped); size ids/codes from list_offsets[nlist]
 * (call once with only list_offsets first). */
int hipann_ivf_export(void *index, float *centroids, int64_t *list_offsets, int64_t *ids, float *codes,
                      char *err_buf, int err_len);

/* List-scan distance form.  HIPANN_IVF_FORM_DECOMPOSED: ‖q‖² + ‖x‖² − 2·q·x clamped ≥ 0
 * (IP: q·x), with ‖x‖² stored per row — the form faiss-metal's IVF path and FAISS's GPU IVFFlat use
 * (MetalIndexIVFFlat.mm:305-318), computed on the fp32 matrix cores (exact fp32 products, fp32
 * accumulation).  HIPANN_IVF_FORM_DIRECT: Σ(q−x)², the form of FAISS's CPU IndexIVFFlat scanner
 * (subtract + FMA per dimension, VALU).  HIPANN_IVF_FORM_DECOMPOSED_VALU: the decomposed form on the
 * VALU kernel (kept for A/B measurement).  All run on the GPU; the decomposed forms need d % 4 == 0
 * and 16-B aligned data and fall back to the direct kernel otherwise.  Returns 0, or −1 for a bad
 * handle / form. */
#define HIPANN_IVF_FORM_DECOMPOSED 0
#define HIPANN_IVF_FORM_DIRECT 1
#define HIPANN_IVF_FORM_DECOMPOSED_VALU 2
/* HIPANN_IVF_FORM_SPLIT3: the decomposed form with q·x on the bf16 matrix cores over a 3-term bf16 split
 * of both operands (six cross products, fp32-level per product, fp32 accumulation);
 * HIPANN_IVF_FORM_SPLIT2: a 2-term split (three products, ≈2^-16 relative per product). */
#define HIPANN_IVF_FORM_SPLIT3 3
#define HIPANN_IVF_FORM_SPLIT2 4
/* HIPANN_IVF_FORM_SPLIT2_EXACT: the SPLIT2 scan keeps the 16 best rows per list only as a
 * filter; every returned distance is recomputed in the direct form Σ(q−x)² (IP: q·x) in fp32, ordered by
 * (distance, label), and a per-query bound (|scan key − exact| ≤ 2^-12·(‖q‖² + max‖x‖²)) proves that no
 * pruned row could enter the top-k — queries that fail it are re-run ON THE DEVICE over their probe lists
 * in the direct form (ivf_fallback_query: one block per flagged query, grid bounded by the device flag count, no host
 * readback), so the call stays asynchronous.  k ≤ 12 (larger k: SPLIT3). */
#define HIPANN_IVF_FORM_SPLIT2_EXACT 5
/* HIPANN_IVF_FORM_HALF_EXACT (default): the same filter + exact rerank, the scan reading a tiled fp16
 * image of the rows (built once: x·2^s, round to nearest even, half the bytes of the fp32 forms) against
 * 2-term fp16 queries on the fp16 matrix cores; the bound is the Cauchy-Schwarz bound of the measured
 * residuals (largest row ‖x − x̂‖, the query's split residual) plus fp32 accumulation.  Codes with a
 * non-finite entry take SPLIT2_EXACT; k ≤ 12 (larger k: SPLIT3).  Results equal SPLIT2_EXACT's. */
#define HIPANN_IVF_FORM_HALF_EXACT 6
/* HIPANN_IVF_FORM_I8_EXACT (opt-in): the same filter + exact rerank over a tiled int8 image (one scale per row,
 * max|x|/127: a quarter of the fp32 rows' bytes) against int8 queries on the int8 matrix cores (exact int32 sums);
 * the scan always keeps per-wave sub-lists and the rerank takes 64 candidates, certified with the int8 residuals.
 * The image is rebuilt at the first search after an add.  Codes with a non-finite entry, or k > 64, take
 * SPLIT2_EXACT.  Results equal SPLIT2_EXACT's. */
#define HIPANN_IVF_FORM_I8_EXACT 7
int hipann_ivf_set_form(void *index, int form);
int hipann_ivf_get_form(void *index);
/* Queries the exact forms' bound check flagged since the index was created (each re-run on the device in
 * the direct form; reading the device-side count synchronises the device). */
int64_t hipann_ivf_rerank_fallbacks(void *index);

/* ---------------------------------------------------------------------------------------------
 * Common
 * ------------------------------------------------------------------------------------------- */

int64_t hipann_ntotal(void *index);
int hipann_dim(void *index);
int hipann_metric(void *index);
/* Bytes of HBM held by the index (vectors + norms + lists). */
int64_t hipann_memory_bytes(void *index);
void hipann_free(void *index);

/* Enable (1) / disable (0) HIP-event timing of the kernels inside each search call. */
int hipann_set_kernel_timing(void *index, int on);

/* Average device time (ms) of the dominant kernel over the last `hipann_*_search*` call, measured
 * with HIP events on the handle's stream (0 if unknown).  `which`: 0 = main scan/GEMM kernel,
 * 1 = merge kernel.  Used by bench.py for the roofline line. */
double hipann_last_kernel_ms(void *index, int which);

#ifdef __cplusplus
}
#endif

#endif /* HIP_ANN_H */
