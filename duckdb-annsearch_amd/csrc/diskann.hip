// diskann.hip — DiskANN batch-distance bridge for gfx950 (include/hip_diskann_bridge.h).
//
// Replaces src/metal_diskann_bridge.mm (:155-253 single query, :255-323 multi query) and the Metal
// kernels faiss-metal/shaders/diskann_distance.metal:15-194 (one 32-lane simdgroup per candidate).
// Semantics: metric 0 → Σ(q−c)², metric 1 → −Σ q·c  (rust_lib/src/distance.rs:15-24).
//
// Kernels
//   dist_rows      — candidates as contiguous fp32 rows (the reference ABI: the caller gathered
//                    them on the host).  One wave per candidate, float4 loads, query chunks from
//                    L1/L2 (consecutive candidates share a query: query_map is grouped per query by
//                    the lock-step BFS, disk_provider.rs:556-577).
//   dist_ids_f32   — HBM-resident fp32 database, candidate = row id (gather).  One wave per row.
//   dist_ids_sq8   — HBM-resident SQ8 codes (provider.rs:161-210), half a wave per row, 16 codes per
//                    lane-load; dequantised as v = code·(scale/255) + min (one fma; within 1 ulp of the
//                    reference's (code/255)·scale + min).
//
// Host side: per-thread stream + staging (thread-safe, unlike the Metal bridge's shared ring,
// metal_diskann_bridge.mm:52-53), a registry of HBM databases, and diskann_hip_search_batch — the
// lock-step best-first BFS of DiskProvider::search_batch (disk_provider.rs:470-652) whose per-step
// distances go through the id-gather kernel.
#include "../../include/hip_diskann_bridge.h"
#include "common.hpp"
#include "runtime.hpp"

#include <algorithm>
#include <cfloat>
#include <cstring>
#include <queue>
#include <unordered_set>
#include <vector>

namespace hipann {

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
}

// candidates: total_n rows of d floats; qmap == nullptr → every candidate uses query 0.
template <bool IP, bool VEC4>
__global__ void __launch_bounds__(256) dist_rows(const float *__restrict__ queries, const float *__restrict__ cands,
                                                 const unsigned *__restrict__ qmap, int total_n, int d,
                                                 float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= total_n) return;
    const unsigned qi = qmap ? qmap[w] : 0u;
    const float *q = queries + (int64_t)qi * d;
    const float *c = cands + w * (int64_t)d;
    float s = 0.f;
    if (VEC4) {
        const float4 *q4 = reinterpret_cast<const float4 *>(q);
        const float4 *c4 = reinterpret_cast<const float4 *>(c);
        for (int j = lane; j < (d >> 2); j += 64) {
            const float4 a = q4[j], b = c4[j];
            if (IP) {
                s = fmaf(a.x, b.x, s); s = fmaf(a.y, b.y, s); s = fmaf(a.z, b.z, s); s = fmaf(a.w, b.w, s);
            } else {
                float t;
                t = a.x - b.x; s = fmaf(t, t, s);
                t = a.y - b.y; s = fmaf(t, t, s);
                t = a.z - b.z; s = fmaf(t, t, s);
                t = a.w - b.w; s = fmaf(t, t, s);
            }
        }
    } else {
        for (int j = lane; j < d; j += 64) {
            if (IP) s = fmaf(q[j], c[j], s);
            else { const float t = q[j] - c[j]; s = fmaf(t, t, s); }
        }
    }
    s = wave_sum(s);
    if (lane == 0) out[w] = IP ? -s : s;
}

template <bool IP, bool VEC4>
__global__ void __launch_bounds__(256) dist_ids_f32(const float *__restrict__ queries, const float *__restrict__ db,
                                                    const unsigned *__restrict__ ids, const unsigned *__restrict__ qmap,
                                                    int total_n, int d, float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= total_n) return;
    const float *q = queries + (int64_t)qmap[w] * d;
    const float *c = db + (int64_t)ids[w] * d;
    float s = 0.f;
    if (VEC4) {
        const float4 *q4 = reinterpret_cast<const float4 *>(q);
        const float4 *c4 = reinterpret_cast<const float4 *>(c);
        for (int j = lane; j < (d >> 2); j += 64) {
            const float4 a = q4[j], b = c4[j];
            if (IP) {
                s = fmaf(a.x, b.x, s); s = fmaf(a.y, b.y, s); s = fmaf(a.z, b.z, s); s = fmaf(a.w, b.w, s);
            } else {
                float t;
                t = a.x - b.x; s = fmaf(t, t, s);
                t = a.y - b.y; s = fmaf(t, t, s);
                t = a.z - b.z; s = fmaf(t, t, s);
                t = a.w - b.w; s = fmaf(t, t, s);
            }
        }
    } else {
        for (int j = lane; j < d; j += 64) {
            if (IP) s = fmaf(q[j], c[j], s);
            else { const float t = q[j] - c[j]; s = fmaf(t, t, s); }
        }
    }
    s = wave_sum(s);
    if (lane == 0) out[w] = IP ? -s : s;
}

// SQ8: half-wave (32 lanes) per candidate, 16 codes (one uint4) per lane per step.  `ab` holds
// per-dimension (scale/255, min) pairs in LDS.  Requires d % 16 == 0 (host checks; otherwise the
// scalar path below).
template <bool IP>
__global__ void __launch_bounds__(256) dist_ids_sq8(const float *__restrict__ queries, const uint8_t *__restrict__ codes,
                                                    const float2 *__restrict__ ab_g, const unsigned *__restrict__ ids,
                                                    const unsigned *__restrict__ qmap, int total_n, int d,
                                                    float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float2 ab[];
    for (int j = threadIdx.x; j < d; j += 256) ab[j] = ab_g[j];
    __syncthreads();
    const int hl = threadIdx.x & 31;
    const int64_t c = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    const bool valid = c < total_n;
    float s = 0.f;
    if (valid) {
        const float *q = queries + (int64_t)qmap[c] * d;
        const uint8_t *row = codes + (int64_t)ids[c] * d;
        for (int j0 = hl * 16; j0 < d; j0 += 32 * 16) {
            const uint4 raw = *reinterpret_cast<const uint4 *>(row + j0);
            const unsigned wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float4 qv = *reinterpret_cast<const float4 *>(q + j0 + 4 * e);
                const float qa[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const float code = (float)((wv[e] >> (8 * b)) & 0xffu);
                    const float2 p = ab[j0 + 4 * e + b];
                    const float v = fmaf(code, p.x, p.y);
                    if (IP) s = fmaf(qa[b], v, s);
                    else { const float t = qa[b] - v; s = fmaf(t, t, s); }
                }
            }
        }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (valid && hl == 0) out[c] = IP ? -s : s;
}

template <bool IP>
__global__ void __launch_bounds__(256) dist_ids_sq8_scalar(const float *__restrict__ queries,
                                                           const uint8_t *__restrict__ codes,
                                                           const float2 *__restrict__ ab, const unsigned *__restrict__ ids,
                                                           const unsigned *__restrict__ qmap, int total_n, int d,
                                                           float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= total_n) return;
    const float *q = queries + (int64_t)qmap[w] * d;
    const uint8_t *row = codes + (int64_t)ids[w] * d;
    float s = 0.f;
    for (int j = lane; j < d; j += 64) {
        const float2 p = ab[j];
        const float v = fmaf((float)row[j], p.x, p.y);
        if (IP) s = fmaf(q[j], v, s);
        else { const float t = q[j] - v; s = fmaf(t, t, s); }
    }
    s = wave_sum(s);
    if (lane == 0) out[w] = IP ? -s : s;
}

// ------------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------------
namespace {

int g_avail = -1;

bool device_ok() {
    if (g_avail < 0) {
        int n = 0;
        g_avail = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
    }
    return g_avail == 1;
}

// Per-thread stream and staging (each calling thread owns its buffers).
struct ThreadCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    DevBuf q, c, m, ids, out;
    HostBuf hq, hc, hm, hids, hout;
    ~ThreadCtx() {
        if (stream) { (void)hipStreamDestroy(stream); }
    }
    void init() {
        int dev = 0;
        HIPANN_CHECK(hipGetDevice(&dev));
        if (stream && dev == device) return;
        if (stream) (void)hipStreamDestroy(stream);
        device = dev;
        HIPANN_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }
};

thread_local ThreadCtx t_ctx;

void launch_rows(const float *q, const float *c, const unsigned *m, int total_n, int d, int metric, float *out,
                 hipStream_t st) {
    const bool v4 = (d % 4 == 0) && ((uintptr_t)q % 16 == 0) && ((uintptr_t)c % 16 == 0);
    dim3 grid((unsigned)ceil_div(total_n, 4)), block(256);
    if (metric == kIP) {
        if (v4) hipLaunchKernelGGL((dist_rows<true, true>), grid, block, 0, st, q, c, m, total_n, d, out);
        else hipLaunchKernelGGL((dist_rows<true, false>), grid, block, 0, st, q, c, m, total_n, d, out);
    } else {
        if (v4) hipLaunchKernelGGL((dist_rows<false, true>), grid, block, 0, st, q, c, m, total_n, d, out);
        else hipLaunchKernelGGL((dist_rows<false, false>), grid, block, 0, st, q, c, m, total_n, d, out);
    }
    HIPANN_CHECK(hipGetLastError());
}

struct DiskDB {
    int device = 0;
    int64_t n = 0;
    int dim = 0;
    int fmt = DISKANN_HIP_FMT_F32;
    DevBuf data;  // fp32 rows or u8 codes
    DevBuf ab;    // float2 per dim (SQ8)
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevBuf q, ids, m, out;
    HostBuf hids, hm, hout;
    KernelTimer timer;
    ~DiskDB() {
        if (stream) { DeviceGuard g(device); (void)hipStreamDestroy(stream); }
    }
};

void launch_ids(DiskDB &db, const float *q, const unsigned *ids, const unsigned *m, int total_n, int metric,
                float *out, hipStream_t st) {
    if (total_n <= 0) return;
    const int d = db.dim;
    if (db.fmt == DISKANN_HIP_FMT_F32) {
        const float *x = db.data.get<float>();
        const bool v4 = (d % 4 == 0) && ((uintptr_t)q % 16 == 0);
        dim3 grid((unsigned)ceil_div(total_n, 4)), block(256);
        if (metric == kIP) {
            if (v4) hipLaunchKernelGGL((dist_ids_f32<true, true>), grid, block, 0, st, q, x, ids, m, total_n, d, out);
            else hipLaunchKernelGGL((dist_ids_f32<true, false>), grid, block, 0, st, q, x, ids, m, total_n, d, out);
        } else {
            if (v4) hipLaunchKernelGGL((dist_ids_f32<false, true>), grid, block, 0, st, q, x, ids, m, total_n, d, out);
            else hipLaunchKernelGGL((dist_ids_f32<false, false>), grid, block, 0, st, q, x, ids, m, total_n, d, out);
        }
    } else {
        const uint8_t *x = db.data.get<uint8_t>();
        const float2 *ab = db.ab.get<float2>();
        if (d % 16 == 0 && (uintptr_t)q % 16 == 0 && d * sizeof(float2) <= 64 * 1024) {
            dim3 grid((unsigned)ceil_div(total_n, 8)), block(256);
            const size_t smem = (size_t)d * sizeof(float2);
            if (metric == kIP) hipLaunchKernelGGL(dist_ids_sq8<true>, grid, block, smem, st, q, x, ab, ids, m, total_n, d, out);
            else hipLaunchKernelGGL(dist_ids_sq8<false>, grid, block, smem, st, q, x, ab, ids, m, total_n, d, out);
        } else {
            dim3 grid((unsigned)ceil_div(total_n, 4)), block(256);
            if (metric == kIP) hipLaunchKernelGGL(dist_ids_sq8_scalar<true>, grid, block, 0, st, q, x, ab, ids, m, total_n, d, out);
            else hipLaunchKernelGGL(dist_ids_sq8_scalar<false>, grid, block, 0, st, q, x, ab, ids, m, total_n, d, out);
        }
    }
    HIPANN_CHECK(hipGetLastError());
}

void set_err(char *buf, int len, const char *msg) {
    if (!buf || len <= 0) return;
    std::strncpy(buf, msg, (size_t)len - 1);
    buf[len - 1] = '\0';
}

// ---- lock-step BFS (DiskProvider::search_batch, disk_provider.rs:470-652) ----
struct Cand {
    float d;
    uint32_t id;
};
struct CandGreater {  // min-heap on (d, id): BinaryHeap<Reverse<(FloatOrd, u32)>>
    bool operator()(const Cand &a, const Cand &b) const { return a.d > b.d || (a.d == b.d && a.id > b.id); }
};

// Rust slice::binary_search_by (std ≥ 1.82) with partial_cmp on distance; returns the insert position.
size_t rust_binary_search(const std::vector<Cand> &res, float dist) {
    size_t size = res.size();
    if (size == 0) return 0;
    size_t base = 0;
    while (size > 1) {
        const size_t half = size / 2, mid = base + half;
        base = (res[mid].d > dist) ? base : mid;
        size -= half;
    }
    const float p = res[base].d;
    if (!(p < dist) && !(p > dist)) return base;
    return base + (p < dist ? 1 : 0);
}

struct QState {
    std::unordered_set<uint32_t> visited;
    std::priority_queue<Cand, std::vector<Cand>, CandGreater> cands;
    std::vector<Cand> result;
    bool active = true;
};

// insert_result (disk_provider.rs:656-678)
void insert_result(QState &s, size_t l, float dist, uint32_t nb) {
    if (s.result.size() < l || dist < s.result.back().d) {
        const size_t pos = rust_binary_search(s.result, dist);
        s.result.insert(s.result.begin() + (ptrdiff_t)pos, Cand{dist, nb});
        if (s.result.size() > l) s.result.resize(l);
        s.cands.push(Cand{dist, nb});
    }
}

}  // namespace
}  // namespace hipann

using namespace hipann;

extern "C" {

int diskann_hip_available(void) {
    try {
        return device_ok() ? 1 : 0;
    } catch (...) {
        return 0;
    }
}

int diskann_hip_batch_distances(const float *query, const float *candidates, int n, int dim, int metric,
                                float *out_distances) {
    if (n <= 0 || dim <= 0 || !query || !candidates || !out_distances) return -1;
    if (metric != kL2 && metric != kIP) return -1;
    try {
        if (!device_ok()) return -1;
        ThreadCtx &t = t_ctx;
        t.init();
        const size_t qb = (size_t)dim * 4, cb = (size_t)n * dim * 4, ob = (size_t)n * 4;
        t.q.ensure(qb, t.device);
        t.c.ensure(cb, t.device);
        t.out.ensure(ob, t.device);
        HIPANN_CHECK(hipMemcpyAsync(t.q.p, query, qb, hipMemcpyHostToDevice, t.stream));
        HIPANN_CHECK(hipMemcpyAsync(t.c.p, candidates, cb, hipMemcpyHostToDevice, t.stream));
        launch_rows(t.q.get<float>(), t.c.get<float>(), nullptr, n, dim, metric, t.out.get<float>(), t.stream);
        HIPANN_CHECK(hipMemcpyAsync(out_distances, t.out.p, ob, hipMemcpyDeviceToHost, t.stream));
        HIPANN_CHECK(hipStreamSynchronize(t.stream));
        return 0;
    } catch (...) {
        return -1;
    }
}

int diskann_hip_multi_batch_distances(const float *queries, const float *candidates, const unsigned int *query_map,
                                      int total_n, int nq, int dim, int metric, float *out_distances) {
    if (total_n <= 0 || nq <= 0 || dim <= 0 || !queries || !candidates || !query_map || !out_distances) return -1;
    if (metric != kL2 && metric != kIP) return -1;
    for (int i = 0; i < total_n; ++i)
        if (query_map[i] >= (unsigned)nq) return -1;
    try {
        if (!device_ok()) return -1;
        ThreadCtx &t = t_ctx;
        t.init();
        const size_t qb = (size_t)nq * dim * 4, cb = (size_t)total_n * dim * 4, mb = (size_t)total_n * 4;
        t.q.ensure(qb, t.device);
        t.c.ensure(cb, t.device);
        t.m.ensure(mb, t.device);
        t.out.ensure(mb, t.device);
        HIPANN_CHECK(hipMemcpyAsync(t.q.p, queries, qb, hipMemcpyHostToDevice, t.stream));
        HIPANN_CHECK(hipMemcpyAsync(t.c.p, candidates, cb, hipMemcpyHostToDevice, t.stream));
        HIPANN_CHECK(hipMemcpyAsync(t.m.p, query_map, mb, hipMemcpyHostToDevice, t.stream));
        launch_rows(t.q.get<float>(), t.c.get<float>(), t.m.get<unsigned>(), total_n, dim, metric, t.out.get<float>(),
                    t.stream);
        HIPANN_CHECK(hipMemcpyAsync(out_distances, t.out.p, mb, hipMemcpyDeviceToHost, t.stream));
        HIPANN_CHECK(hipStreamSynchronize(t.stream));
        return 0;
    } catch (...) {
        return -1;
    }
}

// Drop-in aliases of the reference symbol names (metal_diskann_bridge.h:8-23).
int diskann_metal_available(void) { return diskann_hip_available(); }
int diskann_metal_batch_distances(const float *query, const float *candidates, int n, int dim, int metric,
                                  float *out_distances) {
    return diskann_hip_batch_distances(query, candidates, n, dim, metric, out_distances);
}
int diskann_metal_multi_batch_distances(const float *queries, const float *candidates, const unsigned int *query_map,
                                        int total_n, int nq, int dim, int metric, float *out_distances) {
    return diskann_hip_multi_batch_distances(queries, candidates, query_map, total_n, nq, dim, metric, out_distances);
}

void *diskann_hip_register_db(const void *data, int64_t n, int dim, int fmt, const float *sq8_min,
                              const float *sq8_scale) {
    try {
        if (!device_ok() || n < 0 || dim <= 0 || (n > 0 && !data)) return nullptr;
        if (fmt != DISKANN_HIP_FMT_F32 && fmt != DISKANN_HIP_FMT_SQ8) return nullptr;
        if (fmt == DISKANN_HIP_FMT_SQ8 && (!sq8_min || !sq8_scale)) return nullptr;
        auto db = std::make_unique<DiskDB>();
        HIPANN_CHECK(hipGetDevice(&db->device));
        HIPANN_CHECK(hipStreamCreateWithFlags(&db->stream, hipStreamNonBlocking));
        db->n = n;
        db->dim = dim;
        db->fmt = fmt;
        const size_t bytes = (size_t)n * dim * (fmt == DISKANN_HIP_FMT_F32 ? 4 : 1);
        db->data.ensure(bytes + 16, db->device);
        if (bytes) HIPANN_CHECK(hipMemcpyAsync(db->data.p, data, bytes, hipMemcpyHostToDevice, db->stream));
        if (fmt == DISKANN_HIP_FMT_SQ8) {
            std::vector<float> ab((size_t)dim * 2);
            for (int j = 0; j < dim; ++j) {
                ab[2 * j] = sq8_scale[j] / 255.0f;
                ab[2 * j + 1] = sq8_min[j];
            }
            db->ab.ensure(ab.size() * 4, db->device);
            HIPANN_CHECK(hipMemcpyAsync(db->ab.p, ab.data(), ab.size() * 4, hipMemcpyHostToDevice, db->stream));
        }
        HIPANN_CHECK(hipStreamSynchronize(db->stream));
        return db.release();
    } catch (...) {
        return nullptr;
    }
}

int diskann_hip_multi_batch_distances_ids(void *h, const float *queries, int nq, const unsigned int *ids,
                                          const unsigned int *query_map, int total_n, int metric, float *out) {
    if (!h || !queries || nq <= 0 || total_n < 0 || (total_n > 0 && (!ids || !query_map || !out))) return -1;
    if (metric != kL2 && metric != kIP) return -1;
    auto *db = static_cast<DiskDB *>(h);
    for (int i = 0; i < total_n; ++i)
        if (query_map[i] >= (unsigned)nq || ids[i] >= (uint64_t)db->n) return -1;
    if (total_n == 0) return 0;
    try {
        std::lock_guard<std::mutex> lk(db->mu);
        DeviceGuard g(db->device);
        const size_t qb = (size_t)nq * db->dim * 4, mb = (size_t)total_n * 4;
        db->q.ensure(qb + 16, db->device);
        db->ids.ensure(mb, db->device);
        db->m.ensure(mb, db->device);
        db->out.ensure(mb, db->device);
        HIPANN_CHECK(hipMemcpyAsync(db->q.p, queries, qb, hipMemcpyHostToDevice, db->stream));
        HIPANN_CHECK(hipMemcpyAsync(db->ids.p, ids, mb, hipMemcpyHostToDevice, db->stream));
        HIPANN_CHECK(hipMemcpyAsync(db->m.p, query_map, mb, hipMemcpyHostToDevice, db->stream));
        launch_ids(*db, db->q.get<float>(), db->ids.get<unsigned>(), db->m.get<unsigned>(), total_n, metric,
                   db->out.get<float>(), db->stream);
        HIPANN_CHECK(hipMemcpyAsync(out, db->out.p, mb, hipMemcpyDeviceToHost, db->stream));
        HIPANN_CHECK(hipStreamSynchronize(db->stream));
        return 0;
    } catch (...) {
        return -1;
    }
}

int diskann_hip_multi_batch_distances_ids_device(void *h, const float *queries_dev, int nq, const unsigned int *ids_dev,
                                                 const unsigned int *query_map_dev, int total_n, int metric,
                                                 float *out_dev, void *stream) {
    if (!h || !queries_dev || nq <= 0 || total_n < 0) return -1;
    if (metric != kL2 && metric != kIP) return -1;
    auto *db = static_cast<DiskDB *>(h);
    try {
        DeviceGuard g(db->device);
        hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = the default (null) stream
        ScopedTiming tm(db->timer, st);
        launch_ids(*db, queries_dev, ids_dev, query_map_dev, total_n, metric, out_dev, st);
        return 0;
    } catch (...) {
        return -1;
    }
}

int64_t diskann_hip_db_size(void *h) { return h ? static_cast<DiskDB *>(h)->n : -1; }

void diskann_hip_release_db(void *h) {
    if (!h) return;
    try {
        delete static_cast<DiskDB *>(h);
    } catch (...) {
    }
}

// Lock-step multi-query BFS over an HBM-resident DB (DiskProvider::search_batch semantics, with the
// per-step distance work on the GPU via the id-gather kernel).  adjacency: N × R u32 (u32::MAX pads),
// entry points as in the .diskann header.  Outputs nq × k (ids −1 / dist FLT_MAX past the result).
// stats: [0] distance evaluations, [1] lock-step iterations, [2] GPU calls, [3] reserved.
int diskann_hip_search_batch(void *h, const uint32_t *adj, int R, const uint32_t *eps, int n_ep, const float *queries,
                             int nq, int k, int l_search, int metric, int64_t *out_ids, float *out_d, int64_t *stats,
                             char *eb, int el) {
    try {
        HIPANN_REQUIRE(h && adj && eps && queries && out_ids && out_d, "null argument");
        HIPANN_REQUIRE(R > 0 && nq >= 0 && k > 0, "bad arguments");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 or 1");
        auto *db = static_cast<DiskDB *>(h);
        std::lock_guard<std::mutex> lk(db->mu);
        DeviceGuard g(db->device);
        const uint32_t N = (uint32_t)db->n;
        const int dim = db->dim;
        int64_t nevals = 0, nsteps = 0, ncalls = 0;
        if (nq == 0) {
            if (stats) { stats[0] = stats[1] = stats[2] = stats[3] = 0; }
            return 0;
        }
        const size_t l = (size_t)std::max(l_search, k);
        const hipStream_t st = db->stream;
        // queries resident for the whole search
        db->q.ensure((size_t)nq * dim * 4 + 16, db->device);
        HIPANN_CHECK(hipMemcpyAsync(db->q.p, queries, (size_t)nq * dim * 4, hipMemcpyHostToDevice, st));
        const size_t cap = (size_t)nq * std::max(R, n_ep);
        db->ids.ensure(cap * 4, db->device);
        db->m.ensure(cap * 4, db->device);
        db->out.ensure(cap * 4, db->device);
        db->hids.ensure(cap * 4);
        db->hm.ensure(cap * 4);
        db->hout.ensure(cap * 4);
        uint32_t *hid = db->hids.get<uint32_t>();
        uint32_t *hm = db->hm.get<uint32_t>();
        float *hout = db->hout.get<float>();
        auto gpu_dists = [&](size_t tot) {
            HIPANN_CHECK(hipMemcpyAsync(db->ids.p, hid, tot * 4, hipMemcpyHostToDevice, st));
            HIPANN_CHECK(hipMemcpyAsync(db->m.p, hm, tot * 4, hipMemcpyHostToDevice, st));
            launch_ids(*db, db->q.get<float>(), db->ids.get<unsigned>(), db->m.get<unsigned>(), (int)tot, metric,
                       db->out.get<float>(), st);
            HIPANN_CHECK(hipMemcpyAsync(hout, db->out.p, tot * 4, hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipStreamSynchronize(st));
            nevals += (int64_t)tot;
            ncalls++;
        };
        std::vector<QState> S((size_t)nq);
        // seed entry points (disk_provider.rs:524-538)
        {
            size_t tot = 0;
            for (int qi = 0; qi < nq; ++qi) {
                S[qi].visited.reserve(l * 2);
                for (int e = 0; e < n_ep; ++e) {
                    const uint32_t ep = eps[e];
                    if (S[qi].visited.insert(ep).second && ep < N) {
                        hid[tot] = ep;
                        hm[tot] = (uint32_t)qi;
                        tot++;
                    }
                }
            }
            if (tot) gpu_dists(tot);
            for (size_t i = 0; i < tot; ++i) {
                QState &s = S[hm[i]];
                s.cands.push(Cand{hout[i], hid[i]});
                s.result.push_back(Cand{hout[i], hid[i]});
            }
            for (auto &s : S)
                std::stable_sort(s.result.begin(), s.result.end(), [](const Cand &a, const Cand &b) { return a.d < b.d; });
        }
        for (;;) {
            int active = 0;
            for (auto &s : S) active += s.active ? 1 : 0;
            if (!active) break;
            nsteps++;
            size_t tot = 0;
            for (int qi = 0; qi < nq; ++qi) {
                QState &s = S[qi];
                if (!s.active) continue;
                if (s.cands.empty()) { s.active = false; continue; }
                const Cand c = s.cands.top();
                s.cands.pop();
                if (s.result.size() >= l && c.d > s.result[l - 1].d) { s.active = false; continue; }
                const uint32_t *nbr = adj + (size_t)c.id * R;
                for (int r = 0; r < R; ++r) {
                    const uint32_t nb = nbr[r];
                    if (nb == 0xffffffffu) break;
                    if (nb >= N) continue;
                    if (!s.visited.insert(nb).second) continue;
                    hid[tot] = nb;
                    hm[tot] = (uint32_t)qi;
                    tot++;
                }
            }
            if (!tot) continue;
            gpu_dists(tot);
            for (size_t i = 0; i < tot; ++i) insert_result(S[hm[i]], l, hout[i], hid[i]);
        }
        for (int qi = 0; qi < nq; ++qi) {
            const auto &r = S[qi].result;
            for (int j = 0; j < k; ++j) {
                if ((size_t)j < r.size()) {
                    out_ids[(size_t)qi * k + j] = r[j].id;
                    out_d[(size_t)qi * k + j] = r[j].d;
                } else {
                    out_ids[(size_t)qi * k + j] = -1;
                    out_d[(size_t)qi * k + j] = FLT_MAX;
                }
            }
        }
        if (stats) { stats[0] = nevals; stats[1] = nsteps; stats[2] = ncalls; stats[3] = 0; }
        return 0;
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

}  // extern "C"
