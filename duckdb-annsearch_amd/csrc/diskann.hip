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
//                    lane-load; dequantised bit-identically to the reference, (code/255)·scale + min
//                    (sq8_value).  The resident traversal (diskann_bfs.hip) keeps the fused
//                    (q − min) − code·(scale/255) form, within 1 ulp per element.
//
// Host side: per-thread stream + staging (thread-safe, unlike the Metal bridge's shared ring,
// metal_diskann_bridge.mm:52-53), a registry of HBM databases, and diskann_hip_search_batch — the
// lock-step best-first BFS of DiskProvider::search_batch (disk_provider.rs:470-652) whose per-step
// distances go through the id-gather kernel.
#include "../../include/hip_diskann_bridge.h"
#include "common.hpp"
#include "runtime.hpp"

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cstring>
#include <atomic>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

namespace hipann {

bool diskann_bfs_supported(int d, int fmt, int R, int n_ep, int L, uint32_t N);
void launch_diskann_dup_rows(const uint32_t *adj, int R, int64_t n, uint32_t *dupw, hipStream_t st);
void launch_diskann_bfs(const float *Q, int nq, int d, int fmt, const void *data, const float2 *ab,
                        const uint32_t *adj, const uint32_t *dupw, int R, uint32_t N, const uint32_t *eps, int n_ep, int k, int L,
                        int metric, uint32_t *visited, int64_t vwords, int64_t *out_ids, float *out_d, int *flags,
                        unsigned long long *stats, hipStream_t st);

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

// The host BFS's visited sets on the device (vbits != nullptr): one bit per (query, row), vwords words per query.
// A candidate whose bit was already set (an earlier step of its query, or an earlier slot of the same step) is not
// evaluated: its output is kVisitedBits, a NaN payload no distance arithmetic produces.
constexpr unsigned kVisitedBits = 0x7fc0deadu;
__device__ __forceinline__ bool visit_first(unsigned *vbits, int64_t vwords, unsigned qi, unsigned id) {
    const unsigned bit = 1u << (id & 31u);
    return (atomicOr(vbits + (int64_t)qi * vwords + (id >> 5), bit) & bit) == 0u;
}

template <bool IP, bool VEC4>
__global__ void __launch_bounds__(256) dist_ids_f32(const float *__restrict__ queries, const float *__restrict__ db,
                                                    const unsigned *__restrict__ ids, const unsigned *__restrict__ qmap,
                                                    int total_n, int d, int64_t n, float *__restrict__ out,
                                                    unsigned *__restrict__ vbits, int64_t vwords) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= total_n) return;
    const unsigned id = ids[w];
    if (id >= n) return;  // empty slot of the BFS's fixed per-query layout
    if (vbits) {
        const int first = lane == 0 ? (int)visit_first(vbits, vwords, qmap[w], id) : 0;
        if (!__shfl(first, 0)) {
            if (lane == 0) out[w] = __uint_as_float(kVisitedBits);
            return;
        }
    }
    const float *q = queries + (int64_t)qmap[w] * d;
    const float *c = db + (int64_t)id * d;
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

// SQ8 decode exactly as provider.rs:140-146: (code as f32 / 255.0) * scale + min, two roundings (no fma).
// code/255 is the correctly rounded quotient: q0 = code·fl(1/255), one fma residual step (checked for all
// 256 codes against IEEE division, tests/test_oracle.py).
__device__ __forceinline__ float sq8_value(float code, float scale, float mn) {
    constexpr float r = 1.0f / 255.0f;
    const float q0 = code * r;
    const float a = fmaf(fmaf(-q0, 255.0f, code), r, q0);
    const float b = a * scale;
    return b + mn;
}

// SQ8: a quarter wave (16 lanes) per candidate, 16 codes (one uint4) per lane per unit, every unit of the lane's
// share of the row (d <= 2048: up to 8) issued before any is consumed — 96 code loads of 16 B in flight per wave at
// d 1536, the gather's latency hidden by loads rather than waves.  `ab` holds per-dimension (scale, min) pairs in
// LDS, loaded once per block; blocks loop over groups of 16 candidates.  Requires d % 16 == 0 and d <= 2048 (host
// checks; otherwise the scalar path below).
template <bool IP>
__global__ void __launch_bounds__(256) dist_ids_sq8(const float *__restrict__ queries, const uint8_t *__restrict__ codes,
                                                    const float2 *__restrict__ ab_g, const unsigned *__restrict__ ids,
                                                    const unsigned *__restrict__ qmap, int total_n, int d,
                                                    int64_t n, float *__restrict__ out, unsigned *__restrict__ vbits,
                                                    int64_t vwords, unsigned *__restrict__ done_ctr,
                                                    unsigned *__restrict__ done_tok, unsigned token) {
    extern __shared__ __attribute__((aligned(16))) float2 ab[];
    for (int j = threadIdx.x; j < d; j += 256) ab[j] = ab_g[j];
    __syncthreads();
    const int ql = threadIdx.x & 15;
    for (int64_t c0 = (int64_t)blockIdx.x * 16; c0 < total_n; c0 += (int64_t)gridDim.x * 16) {
        const int64_t c = c0 + (threadIdx.x >> 4);
        const unsigned id = c < total_n ? ids[c] : 0xffffffffu;
        bool valid = id < n;  // also skips empty slots of the BFS's fixed per-query layout
        if (vbits) {  // the candidate's visited bit, by the first lane of its quarter wave
            const int first = valid && ql == 0 ? (int)visit_first(vbits, vwords, qmap[c], id) : 0;
            const bool fresh = __shfl(first, (int)(threadIdx.x & 63) & ~15) != 0;
            if (valid && !fresh && ql == 0) out[c] = __uint_as_float(kVisitedBits);
            valid = valid && fresh;
        }
        float s = 0.f;
        if (valid) {
            const float *q = queries + (int64_t)qmap[c] * d;
            const uint8_t *row = codes + (int64_t)id * d;
            uint4 raws[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j0 = ql * 16 + u * 256;
                if (j0 < d) raws[u] = *reinterpret_cast<const uint4 *>(row + j0);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j0 = ql * 16 + u * 256;
                if (j0 >= d) break;
                const uint4 raw = raws[u];
                const unsigned wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float4 qv = *reinterpret_cast<const float4 *>(q + j0 + 4 * e);
                    const float qa[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const float code = (float)((wv[e] >> (8 * b)) & 0xffu);
                        const float2 p = ab[j0 + 4 * e + b];
                        const float v = sq8_value(code, p.x, p.y);
                        if (IP) s = fmaf(qa[b], v, s);
                        else { const float t = qa[b] - v; s = fmaf(t, t, s); }
                    }
                }
            }
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if (valid && ql == 0) out[c] = IP ? -s : s;
    }
    // done_tok (the host BFS): the launch posts its own completion — every wave's distances (pinned host memory, device
    // mapping) made visible system-wide, the block counted, and the last block to finish writes `token` into the
    // host word the BFS polls — instead of an event recorded behind every step's launch (MI355X_MICROARCH.md,
    // inter-workgroup visibility: release, then the count; the compiler-hazard waits made explicit)
    if (done_tok) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __threadfence_system();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned old = __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (old == gridDim.x - 1) {
                __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
                __threadfence_system();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(done_tok, token, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

template <bool IP>
__global__ void __launch_bounds__(256) dist_ids_sq8_scalar(const float *__restrict__ queries,
                                                           const uint8_t *__restrict__ codes,
                                                           const float2 *__restrict__ ab, const unsigned *__restrict__ ids,
                                                           const unsigned *__restrict__ qmap, int total_n, int d,
                                                           int64_t n, float *__restrict__ out, unsigned *__restrict__ vbits,
                                                           int64_t vwords) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= total_n) return;
    const unsigned id = ids[w];
    if (id >= n) return;
    if (vbits) {
        const int first = lane == 0 ? (int)visit_first(vbits, vwords, qmap[w], id) : 0;
        if (!__shfl(first, 0)) {
            if (lane == 0) out[w] = __uint_as_float(kVisitedBits);
            return;
        }
    }
    const float *q = queries + (int64_t)qmap[w] * d;
    const uint8_t *row = codes + (int64_t)id * d;
    float s = 0.f;
    for (int j = lane; j < d; j += 64) {
        const float2 p = ab[j];
        const float v = sq8_value((float)row[j], p.x, p.y);
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
// host-pointer calls with at most this many candidate bytes run zero-copy from pinned staging
constexpr size_t kZeroCopyMax = (size_t)1 << 20;

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
    DevBuf ab;    // float2 per dim (SQ8): (scale/255, min), the traversal's fused decode
    DevBuf ab_raw;  // float2 per dim (SQ8): (scale, min), the id-gather kernels' exact decode
    hipStream_t stream = nullptr;
    std::mutex mu;
    DevBuf q, ids, m, out;
    HostBuf hids, hm, hout;
    KernelTimer timer;
    // resident graph + BFS scratch (diskann_hip_register_graph / _search_batch_resident)
    int R = 0;
    DevBuf adj_dev, dupw, visited, flags, bstats, eps_dev;
    DevBuf vbits;  // host BFS: the queries' visited bits on the device (one bit per row and query)
    DevBuf bfs_ctr;   // host BFS: per group, the id-gather launch's finished-block count (zero between launches)
    HostBuf bfs_tok;  // host BFS: per group, the token word the launch posts when it is done (polled)
    unsigned bfs_seq = 0;
    std::vector<uint32_t> adj_host;
    ~DiskDB() {
        if (stream) { DeviceGuard g(device); (void)hipStreamDestroy(stream); }
    }
};

// Whether launch_ids posts its own completion token for this DB (the SQ8 vector kernel).
bool ids_post_token(const DiskDB &db, const float *q) {
    return db.fmt != DISKANN_HIP_FMT_F32 && db.dim % 16 == 0 && db.dim <= 2048 && (uintptr_t)q % 16 == 0;
}

void launch_ids(DiskDB &db, const float *q, const unsigned *ids, const unsigned *m, int total_n, int metric,
                float *out, hipStream_t st, unsigned *vbits = nullptr, int64_t vwords = 0, unsigned *done_ctr = nullptr,
                unsigned *done_tok = nullptr, unsigned token = 0) {
    if (total_n <= 0) return;
    const int d = db.dim;
    if (db.fmt == DISKANN_HIP_FMT_F32) {
        const float *x = db.data.get<float>();
        const bool v4 = (d % 4 == 0) && ((uintptr_t)q % 16 == 0);
        dim3 grid((unsigned)ceil_div(total_n, 4)), block(256);
        if (metric == kIP) {
            if (v4) hipLaunchKernelGGL((dist_ids_f32<true, true>), grid, block, 0, st, q, x, ids, m, total_n, d, db.n, out, vbits, vwords);
            else hipLaunchKernelGGL((dist_ids_f32<true, false>), grid, block, 0, st, q, x, ids, m, total_n, d, db.n, out, vbits, vwords);
        } else {
            if (v4) hipLaunchKernelGGL((dist_ids_f32<false, true>), grid, block, 0, st, q, x, ids, m, total_n, d, db.n, out, vbits, vwords);
            else hipLaunchKernelGGL((dist_ids_f32<false, false>), grid, block, 0, st, q, x, ids, m, total_n, d, db.n, out, vbits, vwords);
        }
    } else {
        const uint8_t *x = db.data.get<uint8_t>();
        const float2 *ab = db.ab_raw.get<float2>();
        if (d % 16 == 0 && d <= 2048 && (uintptr_t)q % 16 == 0) {
            // ≤ 8 blocks per CU, each looping over groups of 16 candidates (dist_ids_sq8)
            dim3 grid((unsigned)std::min<int64_t>(ceil_div(total_n, 16), 2048)), block(256);
            const size_t smem = (size_t)d * sizeof(float2);
            if (metric == kIP) hipLaunchKernelGGL(dist_ids_sq8<true>, grid, block, smem, st, q, x, ab, ids, m, total_n, d, db.n, out, vbits, vwords, done_ctr, done_tok, token);
            else hipLaunchKernelGGL(dist_ids_sq8<false>, grid, block, smem, st, q, x, ab, ids, m, total_n, d, db.n, out, vbits, vwords, done_ctr, done_tok, token);
        } else {
            dim3 grid((unsigned)ceil_div(total_n, 4)), block(256);
            if (metric == kIP) hipLaunchKernelGGL(dist_ids_sq8_scalar<true>, grid, block, 0, st, q, x, ab, ids, m, total_n, d, db.n, out, vbits, vwords);
            else hipLaunchKernelGGL(dist_ids_sq8_scalar<false>, grid, block, 0, st, q, x, ab, ids, m, total_n, d, db.n, out, vbits, vwords);
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

// Visited set: open addressing over u32 ids (linear probing, power-of-two capacity, load ≤ 1/2).
// Same membership semantics as the reference's hashbrown::HashSet<u32>; only speed differs.
struct VisitedSet {
    std::vector<uint32_t> slot;  // kEmpty = unused
    uint32_t mask = 0;
    size_t count = 0;
    static constexpr uint32_t kEmpty = 0xffffffffu;
    void init(size_t expect) {
        size_t cap = 64;
        while (cap < 2 * expect) cap <<= 1;
        slot.assign(cap, kEmpty);
        mask = (uint32_t)(cap - 1);
        count = 0;
    }
    static uint32_t hash(uint32_t v) { return (v * 0x9E3779B1u) ^ (v >> 15); }
    void prefetch(uint32_t v) const { __builtin_prefetch(slot.data() + (hash(v) & mask), 1); }
    // Returns true if v was newly inserted (HashSet::insert).  v == kEmpty is stored out of band.
    bool insert(uint32_t v) {
        if (v == kEmpty) {
            const bool fresh = !has_max;
            has_max = true;
            return fresh;
        }
        if (2 * (count + 1) > slot.size()) grow();
        uint32_t i = hash(v) & mask;
        for (;;) {
            const uint32_t x = slot[i];
            if (x == v) return false;
            if (x == kEmpty) { slot[i] = v; ++count; return true; }
            i = (i + 1) & mask;
        }
    }
    bool has_max = false;

  private:
    void grow() {
        std::vector<uint32_t> old;
        old.swap(slot);
        slot.assign(old.size() * 2, kEmpty);
        mask = (uint32_t)(slot.size() - 1);
        for (uint32_t v : old) {
            if (v == kEmpty) continue;
            uint32_t i = hash(v) & mask;
            while (slot[i] != kEmpty) i = (i + 1) & mask;
            slot[i] = v;
        }
    }
};

struct QState {
    VisitedSet visited;
    std::vector<Cand> cands;  // binary min-heap on (d, id) (CandGreater): BinaryHeap<Reverse<..>>
    std::vector<Cand> result;  // sorted by d, at most l entries
    bool active = true;
    int nnew = 0;  // candidates this query put into the current lock-step batch
};

// insert_result (disk_provider.rs:656-678).  (d, id) pairs in `cands` are unique (ids pass the
// visited set once), so any binary heap pops them in the same order as Rust's BinaryHeap.
void insert_result(QState &s, size_t l, float dist, uint32_t nb) {
    if (s.result.size() < l || dist < s.result.back().d) {
        const size_t pos = rust_binary_search(s.result, dist);
        s.result.insert(s.result.begin() + (ptrdiff_t)pos, Cand{dist, nb});
        if (s.result.size() > l) s.result.resize(l);
        s.cands.push_back(Cand{dist, nb});
        std::push_heap(s.cands.begin(), s.cands.end(), CandGreater());
    }
}

// Fork-join pool for the per-step host phases of the lock-step BFS: the calling thread is worker 0,
// the others spin on a generation counter (the phases are ~0.1 ms apart, too short for a futex
// round trip) and exit when the search returns.
class SpinPool {
  public:
    explicit SpinPool(int nthreads) : n_(nthreads < 1 ? 1 : nthreads) {
        for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { worker(t); });
    }
    ~SpinPool() {
        stop_.store(true, std::memory_order_release);
        gen_.fetch_add(1, std::memory_order_acq_rel);
        for (auto &t : th_) t.join();
    }
    int size() const { return n_; }
    // Runs fn(tid) on every worker and returns when all have finished.  Exceptions must not escape fn.
    template <typename F> void run(F &&fn) {
        if (n_ == 1) { fn(0); return; }
        std::function<void(int)> job(fn);
        job_ = &job;
        pending_.store(n_ - 1, std::memory_order_release);
        gen_.fetch_add(1, std::memory_order_acq_rel);
        fn(0);
        while (pending_.load(std::memory_order_acquire) != 0) spin_pause();
        job_ = nullptr;
    }

  private:
    static void spin_pause() { __builtin_ia32_pause(); }
    void worker(int tid) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            int idle = 0;
            while ((g = gen_.load(std::memory_order_acquire)) == seen) {
                spin_pause();
                if (++idle > 4096) { std::this_thread::yield(); idle = 0; }
            }
            seen = g;
            if (stop_.load(std::memory_order_acquire)) return;
            (*job_)(tid);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<bool> stop_{false};
    std::function<void(int)> *job_ = nullptr;
};

int bfs_threads(int nq) {
    int t = 16;  // the GPU box's CPU share per GPU
    if (const char *e = std::getenv("HIPANN_BFS_THREADS")) t = std::atoi(e);
    const int hw = (int)std::thread::hardware_concurrency();
    if (hw > 0) t = std::min(t, hw);
    t = std::min(t, std::max(1, nq / 16));  // ≥ 16 queries per thread
    return std::max(1, t);
}

int bfs_groups(int nq) {
    // two pipelined groups: the GPU gathers one group's distances while the host threads run the other's inserts and
    // expansions (C4 host path, 16 threads: 1 group 34.8K QPS with 9.6 ms of GPU waits per batch, 2 groups 39.9K with
    // 0.5 ms, profiles/r05/diskann_host_bfs_r05.txt); HIPANN_BFS_GROUPS=1..8 for A/B
    int g = 2;
    if (const char *e = std::getenv("HIPANN_BFS_GROUPS")) g = std::atoi(e);
    g = std::min(g, std::max(1, nq / 64));  // ≥ 64 queries per group
    return std::max(1, std::min(g, 8));
}

// Host-driven lock-step BFS (the reference's structure: host state, one id-gather launch per step).
// Caller holds db.mu and the device.  Also the fallback of the resident path for flagged queries.
//
// The queries run in G groups (2 by default), each its own lock-step loop, pipelined: while the GPU gathers group
// g's distances, the host threads insert and expand group g+1's.  A query's trajectory depends only on its own
// state, so grouping changes no result; the batch's step count (the reference's loop iterations) is the largest
// group's.
void host_bfs(DiskDB *db, const uint32_t *adj, int R, const uint32_t *eps, int n_ep, const float *queries, int nq,
              int k, int l_search, int metric, int64_t *out_ids, float *out_d, int64_t *stats) {
    const uint32_t N = (uint32_t)db->n;
    const int dim = db->dim;
    int64_t nevals = 0, nsteps = 0, ncalls = 0;
    if (nq == 0) {
        if (stats) { stats[0] = stats[1] = stats[2] = stats[3] = 0; }
        return;
    }
    const size_t l = (size_t)std::max(l_search, k);
    const hipStream_t st = db->stream;
    // Fixed per-query slot layout: query qi owns slots [qi*S, qi*S + S) of every lock-step batch,
    // S = max(R, n_ep); unused slots hold UINT32_MAX and the kernel skips them.  The query map is
    // therefore constant (uploaded once) and the host phases run per query in parallel with no
    // compaction step.  Per query the candidate order is the reference's (neighbour order).
    const size_t S = (size_t)std::max(R, n_ep);
    const size_t cap = (size_t)nq * S;
    HIPANN_REQUIRE(cap <= (size_t)INT32_MAX, "nq * max(R, n_ep) exceeds INT32_MAX");
    db->q.ensure((size_t)nq * dim * 4 + 16, db->device);
    HIPANN_CHECK(hipMemcpyAsync(db->q.p, queries, (size_t)nq * dim * 4, hipMemcpyHostToDevice, st));
    db->ids.ensure(cap * 4, db->device);
    db->m.ensure(cap * 4, db->device);
    db->out.ensure(cap * 4, db->device);
    db->hids.ensure(cap * 4);
    db->hm.ensure(cap * 4);
    db->hout.ensure(cap * 4);
    uint32_t *hid = db->hids.get<uint32_t>();
    uint32_t *hm = db->hm.get<uint32_t>();
    float *hout = db->hout.get<float>();
    float *hout_dev = static_cast<float *>(host_device_ptr(hout));
    // HIPANN_BFS_ZC_IDS=0 (A/B): the step's ids copied to the device before each gather instead of read in place
    static const bool zc_ids = [] { const char *e = std::getenv("HIPANN_BFS_ZC_IDS"); return !e || std::atoi(e); }();
    const unsigned *hid_dev = static_cast<const unsigned *>(host_device_ptr(hid));
    for (size_t i = 0; i < cap; ++i) hm[i] = (uint32_t)(i / S);
    HIPANN_CHECK(hipMemcpyAsync(db->m.p, hm, cap * 4, hipMemcpyHostToDevice, st));
    std::vector<QState> Sq((size_t)nq);
    // The visited sets live on the device (default): the id-gather kernel sets each candidate's bit and skips the ones
    // already set, so the host phases never probe a per-query hash set (≈ 6K ids, 32-64 KB per query: a cache miss
    // per neighbour).  The host hands over every valid neighbour of the expanded row; an already-visited one comes
    // back as kVisitedBits and is dropped.  HIPANN_BFS_GPU_VISITED=0 (A/B), or more than 1 GiB of bits: the host sets.
    static const bool gv_env = [] { const char *e = std::getenv("HIPANN_BFS_GPU_VISITED"); return !e || std::atoi(e); }();
    const int64_t vwords = ((int64_t)N + 31) / 32;
    const bool gv = gv_env && (int64_t)nq * vwords * 4 <= ((int64_t)1 << 30);
    if (gv) {
        db->vbits.ensure((size_t)nq * vwords * 4, db->device);
        HIPANN_CHECK(hipMemsetAsync(db->vbits.p, 0, (size_t)nq * vwords * 4, st));
    }
    unsigned *vbits = gv ? db->vbits.get<unsigned>() : nullptr;
    auto visited_mark = [](float v) { return __builtin_bit_cast(uint32_t, v) == kVisitedBits; };
    SpinPool pool(bfs_threads(nq));
    const int T = pool.size();
    struct Group {
        int q0 = 0, q1 = 0;
        bool seed = true, done = false, launched = false;
        int64_t steps = 0;
        hipEvent_t ev = nullptr;
        unsigned token = 0;  // the token its last launch posts (tokened launches)
    };
    const int G = bfs_groups(nq);
    // HIPANN_BFS_TOKEN=1 (A/B, measured and rejected in r06): the SQ8 gather posts its own completion (a token word per
    // group in coherent pinned memory, written by the launch's last block) instead of an event recorded behind every
    // step's launch.  Every block must release its distance writes at system scope before it is counted — an L2
    // write-back per block, 2048 per launch — and the C4 host path fell from 71K to 15K QPS (same box, alternating).
    static const bool tok_env = [] { const char *e = std::getenv("HIPANN_BFS_TOKEN"); return e && std::atoi(e); }();
    const bool tok = tok_env && ids_post_token(*db, db->q.get<float>());
    if (tok) {
        if (!db->bfs_ctr.p || db->bfs_ctr.bytes < sizeof(unsigned) * 8) {
            db->bfs_ctr.ensure(sizeof(unsigned) * 8, db->device);
            HIPANN_CHECK(hipMemsetAsync(db->bfs_ctr.p, 0, db->bfs_ctr.bytes, st));
        }
        // coherent pinned memory: the launch's system-scope token store is visible to the polling host at once (the
        // default non-coherent allocation held it back until the stream's end-of-kernel release: 5x slower batches)
        if (db->bfs_tok.ensure(sizeof(unsigned) * 8, hipHostMallocCoherent))
            std::memset(db->bfs_tok.p, 0, sizeof(unsigned) * 8);
    }
    unsigned *tok_dev = tok ? static_cast<unsigned *>(host_device_ptr(db->bfs_tok.p)) : nullptr;
    const volatile unsigned *tok_host = tok ? db->bfs_tok.get<unsigned>() : nullptr;
    std::vector<Group> grp((size_t)G);
    for (int g = 0; g < G; ++g) {
        grp[g].q0 = (int)((int64_t)nq * g / G);
        grp[g].q1 = (int)((int64_t)nq * (g + 1) / G);
        HIPANN_CHECK(hipEventCreateWithFlags(&grp[g].ev, hipEventDisableTiming));
    }
    struct EvFree {
        std::vector<Group> &g;
        ~EvFree() { for (auto &x : g) if (x.ev) (void)hipEventDestroy(x.ev); }
    } ev_free{grp};
    // the group's slots with work (up to its last query with new candidates) through the id-gather kernel
    auto launch = [&](Group &g) {
        int last = g.q0;
        int64_t tot = 0;
        for (int qi = g.q0; qi < g.q1; ++qi)
            if (Sq[qi].nnew) { last = qi + 1; tot += Sq[qi].nnew; }
        g.launched = tot > 0;
        if (!tot) return;
        const size_t o = (size_t)g.q0 * S, span = (size_t)(last - g.q0) * S;
        // zc_ids: the kernel reads the step's ids straight from the pinned host buffer (its device mapping) instead of
        // a host-to-device copy ahead of it (a DMA operation the kernel waits behind, per step)
        if (!zc_ids)
            HIPANN_CHECK(hipMemcpyAsync(db->ids.get<unsigned>() + o, hid + o, span * 4, hipMemcpyHostToDevice, st));
        {
            // the distances go straight into the pinned host buffer through its device mapping (posted writes: no
            // device-to-host copy and its round trip per step)
            ScopedTiming tm(db->timer, st);
            const int gi = (int)(&g - grp.data());
            if (tok) g.token = ++db->bfs_seq == 0 ? ++db->bfs_seq : db->bfs_seq;  // never 0 (the words start at 0)
            launch_ids(*db, db->q.get<float>(), (zc_ids ? hid_dev : db->ids.get<unsigned>()) + o,
                       db->m.get<unsigned>() + o, (int)span, metric, hout_dev + o, st, vbits, vwords,
                       tok ? db->bfs_ctr.get<unsigned>() + gi : nullptr, tok ? tok_dev + gi : nullptr, g.token);
        }
        if (!tok) HIPANN_CHECK(hipEventRecord(g.ev, st));
        ncalls++;
        if (!gv) nevals += tot;  // (gv: the first visits, counted as the phases read them)
    };
    // seed entry points (disk_provider.rs:524-538)
    pool.run([&](int t) {
        const int q0 = (int)((int64_t)nq * t / T), q1 = (int)((int64_t)nq * (t + 1) / T);
        for (int qi = q0; qi < q1; ++qi) {
            QState &s = Sq[qi];
            if (!gv) s.visited.init(std::max<size_t>(l * 2, 1024));
            s.cands.reserve(l * 2);
            s.result.reserve(l + 1);
            uint32_t *slot = hid + (size_t)qi * S;
            int cnt = 0;
            for (int e = 0; e < n_ep; ++e) {
                const uint32_t ep = eps[e];
                if (gv ? ep < N : (s.visited.insert(ep) && ep < N)) slot[cnt++] = ep;
            }
            for (size_t j = (size_t)cnt; j < S; ++j) slot[j] = 0xffffffffu;
            s.nnew = cnt;
        }
    });
    for (auto &g : grp) launch(g);
    // One host phase of a group: the results of its last GPU call (the seeds' into cands + result; later steps'
    // through insert_result), then the loop head (disk_provider.rs:545-652): pop, stop rule, expansion.
    // Returns the loop-head active count.
    std::vector<int64_t> red((size_t)T * 8, 0);  // per-thread head counts, padded against false sharing
    // HIPANN_BFS_CHUNK (A/B): queries per work item taken from a shared counter (default 0: a static 1/T range per
    // thread — measured r05: 8-query chunks 27.6 ms of phases per batch against 19.7 static, 2-query chunks 38 ms: a
    // query's state stays in one core's caches only when the same thread keeps it)
    static const int chunk = [] { const char *e = std::getenv("HIPANN_BFS_CHUNK"); return e ? std::atoi(e) : 0; }();
    std::atomic<int> next_q{0};
    auto phase = [&](Group &g) {
        const int n = g.q1 - g.q0;
        const bool seed = g.seed;
        next_q.store(g.q0, std::memory_order_relaxed);
        pool.run([&](int t) {
            int64_t head = 0, evals = 0;
            int q0, q1;
            if (chunk > 0) {
                q0 = next_q.fetch_add(chunk, std::memory_order_relaxed);
                q1 = std::min(q0 + chunk, g.q1);
            } else {
                q0 = g.q0 + (int)((int64_t)n * t / T);
                q1 = g.q0 + (int)((int64_t)n * (t + 1) / T);
            }
            for (; q0 < g.q1; ) {
            for (int qi = q0; qi < q1; ++qi) {
                QState &s = Sq[qi];
                uint32_t *slot = hid + (size_t)qi * S;
                const float *dd = hout + (size_t)qi * S;
                if (seed) {
                    for (int j = 0; j < s.nnew; ++j) {
                        if (gv && visited_mark(dd[j])) continue;  // a repeated entry point
                        ++evals;
                        s.cands.push_back(Cand{dd[j], slot[j]});
                        std::push_heap(s.cands.begin(), s.cands.end(), CandGreater());
                        s.result.push_back(Cand{dd[j], slot[j]});
                    }
                    std::stable_sort(s.result.begin(), s.result.end(),
                                     [](const Cand &x, const Cand &y) { return x.d < y.d; });
                } else {
                    for (int j = 0; j < s.nnew; ++j) {
                        if (gv && visited_mark(dd[j])) continue;
                        ++evals;
                        insert_result(s, l, dd[j], slot[j]);
                    }
                }
                const int prev = s.nnew;  // slots >= prev are already empty
                s.nnew = 0;
                head += s.active ? 1 : 0;  // the reference's loop-head active count
                if (s.active) {
                    if (s.cands.empty()) {
                        s.active = false;
                    } else {
                        std::pop_heap(s.cands.begin(), s.cands.end(), CandGreater());
                        const Cand c = s.cands.back();
                        s.cands.pop_back();
                        if (s.result.size() >= l && c.d > s.result[l - 1].d) {
                            s.active = false;
                        } else {
                            const uint32_t *nbr = adj + (size_t)c.id * R;
                            if (gv) {  // every valid neighbour: the device keeps the visited sets
                                int cnt = 0;
                                for (int r = 0; r < R; ++r) {
                                    const uint32_t nb = nbr[r];
                                    if (nb == 0xffffffffu) break;  // get_neighbors trims at the first sentinel
                                    if (nb < N) slot[cnt++] = nb;
                                }
                                s.nnew = cnt;
                            } else {
                            // the row's valid neighbours first, with their visited-set slots prefetched: the set
                            // (≈ 6K ids, 32-64 KB per query) misses cache on nearly every probe, and 64 overlapped
                            // misses cost about one
                            uint32_t nv[256];
                            int cnt = 0;
                            bool end = false;
                            for (int r0 = 0; r0 < R && !end; r0 += 256) {  // (rows wider than 256 in pieces)
                                int m = 0;
                                for (int r = r0; r < R && r < r0 + 256; ++r) {
                                    const uint32_t nb = nbr[r];
                                    if (nb == 0xffffffffu) {  // get_neighbors trims at the first sentinel
                                        end = true;
                                        break;
                                    }
                                    if (nb >= N) continue;
                                    nv[m++] = nb;
                                    s.visited.prefetch(nb);
                                }
                                for (int j = 0; j < m; ++j)
                                    if (s.visited.insert(nv[j])) slot[cnt++] = nv[j];
                            }
                            s.nnew = cnt;
                            }
                        }
                    }
                }
                for (int j = s.nnew; j < prev; ++j) slot[j] = 0xffffffffu;
                // the adjacency row the next pop most likely takes (the heap's top now; the next step's inserts rarely
                // change it), into cache while the GPU computes this step's distances
                if (s.active && !s.cands.empty()) __builtin_prefetch(adj + (size_t)s.cands.front().id * R);
            }
            if (chunk <= 0) break;
            q0 = next_q.fetch_add(chunk, std::memory_order_relaxed);
            q1 = std::min(q0 + chunk, g.q1);
            }
            red[(size_t)t * 8] = head;
            red[(size_t)t * 8 + 1] = evals;
        });
        g.seed = false;
        int64_t head = 0;
        for (int t = 0; t < T; ++t) {
            head += red[(size_t)t * 8];
            if (gv) nevals += red[(size_t)t * 8 + 1];
        }
        return head;
    };
    // HIPANN_BFS_PROF=1 (tuning): host time in the GPU waits, the host phases and the launches, on stderr
    static const bool prof = std::getenv("HIPANN_BFS_PROF") != nullptr;
    using clk = std::chrono::steady_clock;
    double t_wait = 0, t_phase = 0, t_launch = 0;
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); };
    const auto t_all = clk::now();
    for (int live = G; live > 0;) {
        for (auto &g : grp) {
            if (g.done) continue;
            auto t0 = clk::now();
            if (g.launched) {
                if (tok) wait_posted(tok_host + (&g - grp.data()), g.token, st);
                else wait_event(g.ev);
            }
            auto t1 = clk::now();
            const int64_t head = phase(g);
            auto t2 = clk::now();
            if (prof) {
                t_wait += std::chrono::duration<double, std::micro>(t1 - t0).count();
                t_phase += std::chrono::duration<double, std::micro>(t2 - t1).count();
            }
            if (!head) {
                g.done = true;
                --live;
                continue;
            }
            g.steps++;
            launch(g);  // (nothing when no query of the group expanded new neighbours)
            if (prof) t_launch += since(t2);
        }
    }
    if (prof)
        std::fprintf(stderr, "hipann bfs: nq %d groups %d threads %d calls %lld: total %.0f us, waits %.0f, phases %.0f, "
                             "launches %.0f\n", nq, G, T, (long long)ncalls, since(t_all), t_wait, t_phase, t_launch);
    for (auto &g : grp) nsteps = std::max(nsteps, g.steps);
    for (int qi = 0; qi < nq; ++qi) {
        const auto &r = Sq[qi].result;
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
        if (cb <= kZeroCopyMax) {
            // small calls (the per-step shapes of metal_ffi.rs): stage into this thread's pinned buffers
            // and let the kernel read / write them over PCIe — no DMA round trips (the reference's
            // zero-copy wrap of page-aligned buffers, metal_diskann_bridge.mm:182-222)
            t.hq.ensure(qb);
            t.hc.ensure(cb);
            t.hout.ensure(ob);
            std::memcpy(t.hq.p, query, qb);
            std::memcpy(t.hc.p, candidates, cb);
            void *dq = nullptr, *dc = nullptr, *dout = nullptr;
            HIPANN_CHECK(hipHostGetDevicePointer(&dq, t.hq.p, 0));
            HIPANN_CHECK(hipHostGetDevicePointer(&dc, t.hc.p, 0));
            HIPANN_CHECK(hipHostGetDevicePointer(&dout, t.hout.p, 0));
            launch_rows(static_cast<const float *>(dq), static_cast<const float *>(dc), nullptr, n, dim, metric,
                        static_cast<float *>(dout), t.stream);
            HIPANN_CHECK(hipStreamSynchronize(t.stream));
            std::memcpy(out_distances, t.hout.p, ob);
            return 0;
        }
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
            // ab: (scale/255, min) for the traversal's fused form; ab_raw: (scale, min) for the id-gather
            // kernels' exact decode
            std::vector<float> ab((size_t)dim * 2), abr((size_t)dim * 2);
            for (int j = 0; j < dim; ++j) {
                ab[2 * j] = sq8_scale[j] / 255.0f;
                ab[2 * j + 1] = sq8_min[j];
                abr[2 * j] = sq8_scale[j];
                abr[2 * j + 1] = sq8_min[j];
            }
            db->ab.ensure(ab.size() * 4, db->device);
            db->ab_raw.ensure(abr.size() * 4, db->device);
            HIPANN_CHECK(hipMemcpyAsync(db->ab.p, ab.data(), ab.size() * 4, hipMemcpyHostToDevice, db->stream));
            HIPANN_CHECK(hipMemcpyAsync(db->ab_raw.p, abr.data(), abr.size() * 4, hipMemcpyHostToDevice, db->stream));
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

int diskann_hip_set_kernel_timing(void *h, int on) {
    if (!h) return -1;
    auto *db = static_cast<DiskDB *>(h);
    try {
        std::lock_guard<std::mutex> lk(db->mu);
        db->timer.reset(on != 0, db->device);
        return 0;
    } catch (...) {
        return -1;
    }
}

int diskann_hip_kernel_stats(void *h, double *total_ms, int64_t *launches) {
    if (!h || !total_ms || !launches) return -1;
    auto *db = static_cast<DiskDB *>(h);
    try {
        std::lock_guard<std::mutex> lk(db->mu);
        DeviceGuard g(db->device);
        *launches = (int64_t)db->timer.used;
        *total_ms = db->timer.average_ms() * (double)db->timer.used;
        return 0;
    } catch (...) {
        return -1;
    }
}

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
        RoctxRange rr("hipann.diskann.host_bfs");
        host_bfs(db, adj, R, eps, n_ep, queries, nq, k, l_search, metric, out_ids, out_d, stats);
        return 0;
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

int diskann_hip_register_graph(void *h, const uint32_t *adj, int R) {
    if (!h || !adj || R <= 0) return -1;
    auto *db = static_cast<DiskDB *>(h);
    try {
        std::lock_guard<std::mutex> lk(db->mu);
        DeviceGuard g(db->device);
        const size_t cnt = (size_t)db->n * R;
        db->adj_host.assign(adj, adj + cnt);
        db->adj_dev.ensure(cnt * 4 + 16, db->device);
        if (cnt) HIPANN_CHECK(hipMemcpyAsync(db->adj_dev.p, adj, cnt * 4, hipMemcpyHostToDevice, db->stream));
        // rows with a repeated id (the traversal's first-occurrence dedupe runs only on those)
        if (R <= 64) {  // (wider graphs run on the host BFS)
            db->dupw.ensure((size_t)((db->n + 31) / 32) * 4 + 16, db->device);
            launch_diskann_dup_rows(db->adj_dev.get<uint32_t>(), R, db->n, db->dupw.get<uint32_t>(), db->stream);
        } else {
            db->dupw.release();
        }
        HIPANN_CHECK(hipStreamSynchronize(db->stream));
        db->R = R;
        return 0;
    } catch (...) {
        return -1;
    }
}

// Resident search: queries / outputs in HBM, asynchronous launch on `stream`, then a wait for the
// per-query flags (the rare flagged queries and unsupported shapes go through host_bfs).
int diskann_hip_search_batch_resident_device(void *h, const uint32_t *eps, int n_ep, const float *queries_dev, int nq,
                                             int k, int l_search, int metric, int64_t *out_ids_dev,
                                             float *out_d_dev, int64_t *stats, void *stream, char *eb, int el) {
    RoctxRange r_all("hipann.diskann.resident");
    try {
        HIPANN_REQUIRE(h && (n_ep == 0 || eps) && (nq == 0 || (queries_dev && out_ids_dev && out_d_dev)),
                       "null argument");
        HIPANN_REQUIRE(nq >= 0 && k > 0 && n_ep >= 0, "bad arguments");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 or 1");
        auto *db = static_cast<DiskDB *>(h);
        std::lock_guard<std::mutex> lk(db->mu);
        HIPANN_REQUIRE(db->R > 0, "no graph registered (diskann_hip_register_graph)");
        DeviceGuard g(db->device);
        const hipStream_t st = stream ? static_cast<hipStream_t>(stream) : db->stream;
        if (stats) { stats[0] = stats[1] = stats[2] = stats[3] = 0; }
        if (nq == 0) return 0;
        const uint32_t N = (uint32_t)db->n;
        const int L = std::max(l_search, std::min<int>(k, (int)std::min<int64_t>(db->n, INT32_MAX)));
        const int kk = k;
        std::vector<int> flags((size_t)nq, 0);
        const bool gpu_ok = db->n > 0 && diskann_bfs_supported(db->dim, db->fmt, db->R, n_ep, L, N);
        int64_t gsteps = 0, gevals = 0, gpops = 0;
        if (gpu_ok) {
            const int64_t vwords = ((int64_t)N + 31) / 32;
            // bound the visited bitmaps to ~2 GiB: sub-batches of queries
            const int64_t per = std::max<int64_t>(1, std::min<int64_t>(nq, ((int64_t)2 << 30) / (vwords * 4)));
            db->visited.ensure((size_t)per * vwords * 4, db->device);
            db->flags.ensure((size_t)nq * 4, db->device);
            db->bstats.ensure(80, db->device);
            db->eps_dev.ensure((size_t)std::max(n_ep, 1) * 4, db->device);
            if (n_ep) HIPANN_CHECK(hipMemcpyAsync(db->eps_dev.p, eps, (size_t)n_ep * 4, hipMemcpyHostToDevice, st));
            HIPANN_CHECK(hipMemsetAsync(db->bstats.p, 0, 80, st));
            for (int64_t q0 = 0; q0 < nq; q0 += per) {
                const int64_t qn = std::min<int64_t>(per, nq - q0);
                HIPANN_CHECK(hipMemsetAsync(db->visited.p, 0, (size_t)qn * vwords * 4, st));
                ScopedTiming tm(db->timer, st);
                launch_diskann_bfs(queries_dev + q0 * db->dim, (int)qn, db->dim, db->fmt, db->data.p,
                                   db->ab.get<float2>(), db->adj_dev.get<uint32_t>(), db->dupw.get<uint32_t>(), db->R, N,
                                   db->eps_dev.get<uint32_t>(), n_ep, kk, L, metric, db->visited.get<uint32_t>(),
                                   vwords, out_ids_dev + q0 * kk, out_d_dev + q0 * kk, db->flags.get<int>() + q0,
                                   db->bstats.get<unsigned long long>(), st);
            }
            unsigned long long hs[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            HIPANN_CHECK(hipMemcpyAsync(flags.data(), db->flags.p, (size_t)nq * 4, hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipMemcpyAsync(hs, db->bstats.p, 80, hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipStreamSynchronize(st));
            if (hs[3] + hs[4] + hs[5] + hs[6] + hs[7] + hs[8]) {  // tuning builds (HIPANN_BFS_PROF)
                const double st = (double)std::max<unsigned long long>(hs[2], 1);
                std::fprintf(stderr,
                             "[bfs-prof] wave-0 cycles per step: select %.0f adjacency %.0f dedupe %.0f visited %.0f "
                             "dist %.0f insert %.0f; speculated rows used %.3f\n",
                             hs[3] / st, hs[4] / st, hs[5] / st, hs[6] / st, hs[7] / st, hs[8] / st, hs[9] / st);
            }
            gevals = (int64_t)hs[0];
            gsteps = (int64_t)hs[1];
            gpops = (int64_t)hs[2];
        } else {
            std::fill(flags.begin(), flags.end(), 1);
        }
        // host BFS for flagged queries (exact; queries are independent)
        std::vector<int> redo;
        for (int i = 0; i < nq; ++i)
            if (flags[i]) redo.push_back(i);
        int64_t hsteps = 0, hevals = 0;
        if (!redo.empty()) {
            const int nr = (int)redo.size(), dim = db->dim;
            std::vector<float> qh((size_t)nr * dim);
            for (int j = 0; j < nr; ++j)
                HIPANN_CHECK(hipMemcpyAsync(qh.data() + (size_t)j * dim, queries_dev + (size_t)redo[j] * dim,
                                            (size_t)dim * 4, hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipStreamSynchronize(st));
            std::vector<int64_t> oi((size_t)nr * kk);
            std::vector<float> od((size_t)nr * kk);
            int64_t hst[4] = {0, 0, 0, 0};
            host_bfs(db, db->adj_host.data(), db->R, eps, n_ep, qh.data(), nr, kk, l_search, metric, oi.data(),
                     od.data(), hst);
            for (int j = 0; j < nr; ++j) {
                HIPANN_CHECK(hipMemcpyAsync(out_ids_dev + (size_t)redo[j] * kk, oi.data() + (size_t)j * kk,
                                            (size_t)kk * 8, hipMemcpyHostToDevice, st));
                HIPANN_CHECK(hipMemcpyAsync(out_d_dev + (size_t)redo[j] * kk, od.data() + (size_t)j * kk,
                                            (size_t)kk * 4, hipMemcpyHostToDevice, st));
            }
            HIPANN_CHECK(hipStreamSynchronize(st));
            hevals = hst[0];
            hsteps = hst[1];
        }
        if (stats) {
            stats[0] = gevals + hevals;
            stats[1] = std::max(gsteps, hsteps);
            stats[2] = gpops;
            stats[3] = (int64_t)redo.size();
        }
        return 0;
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

int diskann_hip_search_batch_resident(void *h, const uint32_t *eps, int n_ep, const float *queries, int nq, int k,
                                      int l_search, int metric, int64_t *out_ids, float *out_d, int64_t *stats,
                                      char *eb, int el) {
    try {
        HIPANN_REQUIRE(h && (nq == 0 || (queries && out_ids && out_d)), "null argument");
        HIPANN_REQUIRE(nq >= 0 && k > 0, "bad arguments");
        auto *db = static_cast<DiskDB *>(h);
        DevBuf q, oi, od;
        int dev;
        {
            std::lock_guard<std::mutex> lk(db->mu);
            dev = db->device;
        }
        DeviceGuard g(dev);
        const size_t qb = (size_t)std::max(nq, 1) * db->dim * 4, ob = (size_t)std::max(nq, 1) * k;
        q.ensure(qb, dev);
        oi.ensure(ob * 8, dev);
        od.ensure(ob * 4, dev);
        hipStream_t st;
        HIPANN_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        struct SG { hipStream_t s; ~SG() { (void)hipStreamDestroy(s); } } sg{st};
        if (nq) HIPANN_CHECK(hipMemcpyAsync(q.p, queries, (size_t)nq * db->dim * 4, hipMemcpyHostToDevice, st));
        const int rc = diskann_hip_search_batch_resident_device(h, eps, n_ep, q.get<float>(), nq, k, l_search, metric,
                                                                oi.get<int64_t>(), od.get<float>(), stats, st, eb, el);
        if (rc != 0) return rc;
        if (nq) {
            HIPANN_CHECK(hipMemcpyAsync(out_ids, oi.p, (size_t)nq * k * 8, hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipMemcpyAsync(out_d, od.p, (size_t)nq * k * 4, hipMemcpyDeviceToHost, st));
        }
        HIPANN_CHECK(hipStreamSynchronize(st));
        return 0;
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

}  // extern "C"
