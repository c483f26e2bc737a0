// diskann_bfs.hip — GPU-resident DiskANN beam search (DiskProvider::search_batch on the device).
//
// The reference runs the lock-step best-first search on the host and ships every step's candidate
// vectors to the GPU (rust_lib/src/disk_provider.rs:470-678 → metal_diskann_bridge.mm:255-323): one
// PCIe round trip per step, host hash sets and heaps.  Here the whole traversal of a query runs in
// one wavefront with the database (fp32 rows or SQ8 codes), the adjacency (N × R u32) and a per-query
// visited bitmap resident in HBM.
//
// Exactness.  The wave reproduces the reference's per-query state machine step for step:
//   * result: the sorted list of ≤ L (dist, id), register-resident (element e = s·64 + lane in slot
//     s), insert position by Rust's slice::binary_search_by with partial_cmp (std ≥ 1.82), shift,
//     truncate to L (insert_result, disk_provider.rs:656-678);
//   * candidates: the reference's BinaryHeap<Reverse<(FloatOrd, u32)>> pops the smallest (dist, id).
//     Every heap entry was inserted into `result` when pushed; entries with dist < result[L−1] are
//     still in `result` (truncation only removes the maximum and the threshold never rises), entries
//     with dist > result[L−1] can only be popped as the stopping pop.  So the heap is represented as
//     "result entries not yet expanded" (flag bit 31 of the id) plus a spill list of entries evicted
//     from `result` with dist == the new result[L−1] (exact ties at the boundary, which stay
//     poppable); spill entries that fall above the threshold are dropped.  An empty set then stops
//     the query exactly where the reference pops a candidate worse than result[L−1].
//   * expansion: neighbours up to the first u32::MAX (get_neighbors, :319-331), ids ≥ N skipped, the
//     visited insert in neighbour order (first occurrence wins), distances, then insert_result in
//     neighbour order.
// Distances: L2 Σ(q − v)², IP −Σ q·v (distance.rs:15-24); SQ8 v = code·(scale/255) + min.  The fused
// form here computes (q − min) − code·a in one fma (L2) and −(Σ(q·a)·code + Σ q·min) (IP): within the
// bridge tolerance of the reference's dequantise-then-diff order.
// A query whose spill list overflows (64 boundary ties) is flagged and re-run by the host BFS.
#include "common.hpp"

#include <cfloat>
#include <cstdint>

namespace hipann {
namespace {

constexpr unsigned kNone = 0xffffffffu;
constexpr unsigned kExpanded = 0x80000000u;

__device__ __forceinline__ unsigned ford(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funord(unsigned s) {
    return __uint_as_float((s & 0x80000000u) ? (s & 0x7fffffffu) : ~s);
}
__device__ __forceinline__ float rl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ unsigned rl_u(unsigned v, int l) { return (unsigned)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rl_u64(uint64_t v, int l) {
    return ((uint64_t)rl_u((unsigned)(v >> 32), l) << 32) | rl_u((unsigned)v, l);
}
__device__ __forceinline__ float wsum(float s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    return s;
}
__device__ __forceinline__ uint64_t wmin_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = (uint64_t)__shfl_xor((unsigned long long)v, o);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ float up1_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(((lane - 1) & 63) << 2, __float_as_int(v)));
}
__device__ __forceinline__ unsigned up1_u(unsigned v, int lane) {
    return (unsigned)__builtin_amdgcn_ds_bpermute(((lane - 1) & 63) << 2, (int)v);
}

// dims per 16-byte chunk: 16 SQ8 codes or 4 floats; lane `l`, chunk t covers chunk index l + 64t
template <bool SQ8> struct Fmt {
    static constexpr int kDims = SQ8 ? 16 : 4;
};

template <int S>
struct ResultList {
    float d[S];
    unsigned id[S];  // bit 31 = expanded
    __device__ __forceinline__ float get_d(int e) const {
        const int s = e >> 6;
        float v = d[0];
#pragma unroll
        for (int t = 1; t < S; ++t) if (s == t) v = d[t];
        return rl_f(v, e & 63);
    }
    __device__ __forceinline__ unsigned get_id(int e) const {
        const int s = e >> 6;
        unsigned v = id[0];
#pragma unroll
        for (int t = 1; t < S; ++t) if (s == t) v = id[t];
        return rl_u(v, e & 63);
    }
    // slice::binary_search_by(|p| p.0.partial_cmp(&dist).unwrap_or(Equal)).unwrap_or_else(|e| e)
    __device__ __forceinline__ int rust_pos(float dist, int len) const {
        if (len == 0) return 0;
        int size = len, base = 0;
        while (size > 1) {
            const int half = size >> 1, mid = base + half;
            base = (get_d(mid) > dist) ? base : mid;
            size -= half;
        }
        const float p = get_d(base);
        if (!(p < dist) && !(p > dist)) return base;
        return base + (p < dist ? 1 : 0);
    }
    // insert (dist, nid) at pos (elements ≥ pos move up one; element 64·S − 1 falls off)
    __device__ __forceinline__ void insert_at(int pos, float dist, unsigned nid, int lane) {
#pragma unroll
        for (int s = S - 1; s >= 0; --s) {
            float ud = up1_f(d[s], lane);
            unsigned ui = up1_u(id[s], lane);
            if (s > 0) {
                const float c63 = rl_f(d[s - 1], 63);
                const unsigned i63 = rl_u(id[s - 1], 63);
                if (lane == 0) { ud = c63; ui = i63; }
            }
            const int e = s * 64 + lane;
            if (e == pos) { d[s] = dist; id[s] = nid; }
            else if (e > pos) { d[s] = ud; id[s] = ui; }
        }
    }
    __device__ __forceinline__ void clear_at(int e, int lane) {
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s * 64 + lane == e) { d[s] = __builtin_inff(); id[s] = kNone; }
    }
};

template <int S, int T, bool SQ8, bool IP>
__global__ void __launch_bounds__(64)
diskann_bfs(const float *__restrict__ Qs, int nq, int d, const uint8_t *__restrict__ data,
            const float2 *__restrict__ ab, const uint32_t *__restrict__ adj, int R, uint32_t N,
            const uint32_t *__restrict__ eps, int n_ep, int k, int L, uint32_t *__restrict__ visited,
            int64_t vwords, int64_t *__restrict__ out_ids, float *__restrict__ out_d, int *__restrict__ flags,
            unsigned long long *__restrict__ stats) {
    constexpr int DC = Fmt<SQ8>::kDims;
    constexpr int P = 8 / T;  // rows in flight per distance batch
    const int qi = blockIdx.x;
    if (qi >= nq) return;
    const int lane = threadIdx.x;
    const size_t rowbytes = SQ8 ? (size_t)d : (size_t)d * 4;
    uint32_t *vis = visited + (int64_t)qi * vwords;
    const float *q = Qs + (int64_t)qi * d;

    // per-lane query terms for the lane's dims (chunk t: dims DC·(lane + 64t) ..)
    float qp[T][DC], av[T][DC];
    float cq = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int e = 0; e < DC; ++e) {
            const int dim = DC * (lane + 64 * t) + e;
            float qv = 0.f, a = 0.f, b = 0.f;
            if (dim < d) {
                qv = q[dim];
                if (SQ8) { const float2 p = ab[dim]; a = p.x; b = p.y; }
            }
            if (SQ8) {
                if (IP) { qp[t][e] = qv * a; cq = fmaf(qv, b, cq); }
                else { qp[t][e] = qv - b; }
                av[t][e] = a;
            } else {
                qp[t][e] = qv;
                av[t][e] = 0.f;
            }
        }
    if (SQ8 && IP) cq = wsum(cq);

    auto load_row = [&](uint32_t rid, uint4 (&v)[T]) {
        const uint8_t *base = data + (size_t)rid * rowbytes;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const size_t off = (size_t)16 * (lane + 64 * t);
            v[t] = off < rowbytes ? *reinterpret_cast<const uint4 *>(base + off) : make_uint4(0, 0, 0, 0);
        }
    };
    auto row_dist = [&](const uint4 (&v)[T]) -> float {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const unsigned w[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
            if (SQ8) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float c = (float)((w[e >> 2] >> (8 * (e & 3))) & 0xffu);
                    if (IP) acc = fmaf(qp[t][e], c, acc);
                    else { const float tt = fmaf(-c, av[t][e], qp[t][e]); acc = fmaf(tt, tt, acc); }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = __uint_as_float(w[e]);
                    if (IP) acc = fmaf(qp[t][e], x, acc);
                    else { const float tt = qp[t][e] - x; acc = fmaf(tt, tt, acc); }
                }
            }
        }
        acc = wsum(acc);
        return IP ? -(acc + cq) : acc;
    };
    // distances of the rows named by `nb` on the lanes of mask m (lane-indexed result)
    auto dists = [&](uint64_t m, uint32_t nb) -> float {
        float mine = 0.f;
        while (m) {
            int js[P];
            uint32_t ids[P];
            int cnt = 0;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                js[p] = -1;
                ids[p] = 0;
                if (m) {
                    const int j = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    js[p] = j;
                    ids[p] = rl_u(nb, j);
                    cnt++;
                }
            }
            uint4 v[P][T];
#pragma unroll
            for (int p = 0; p < P; ++p)
                if (p < cnt) load_row(ids[p], v[p]);
#pragma unroll
            for (int p = 0; p < P; ++p)
                if (p < cnt) {
                    const float dd = row_dist(v[p]);
                    if (lane == js[p]) mine = dd;
                }
        }
        return mine;
    };

    ResultList<S> res;
#pragma unroll
    for (int s = 0; s < S; ++s) { res.d[s] = __builtin_inff(); res.id[s] = kNone; }
    int len = 0;
    uint64_t spill = ~0ull;  // lane < nspill: a heap entry evicted from result on a boundary tie
    int nspill = 0;
    int flag = 0;
    unsigned long long evals = 0;
    int steps = 0;

    // ---- seeds (disk_provider.rs:524-538): visited insert in order, distance, push, stable sort ----
    {
        const uint32_t ep = lane < n_ep ? eps[lane] : kNone;
        const bool ok = lane < n_ep && ep < N;
        bool dup = false;
        uint64_t vm = __ballot(ok);
        while (vm) {
            const int i = __ffsll((unsigned long long)vm) - 1;
            vm &= vm - 1;
            if (ok && lane > i && ep == rl_u(ep, i)) dup = true;
        }
        const bool fresh = ok && !dup;
        if (fresh) atomicOr(vis + (ep >> 5), 1u << (ep & 31));
        const uint64_t m = __ballot(fresh);
        evals += __popcll(m);
        const float dd = dists(m, ep);
        // stable sort by distance: key (dist, lane) lexicographic; non-seeds last
        float key = fresh ? dd : __builtin_inff();
        int src = fresh ? lane : 64 + lane;
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const float ok2 = __shfl_xor(key, stride);
                const int os = __shfl_xor(src, stride);
                const bool keep_min = ((lane & stride) == 0) == ((lane & size) == 0);
                const bool o_less = ok2 < key || (ok2 == key && os < src);  // (key, src) pairs are unique
                if (keep_min == o_less) { key = ok2; src = os; }
            }
        len = __popcll(m);
        const uint32_t sid = __shfl(ep, src & 63);
        if (lane < len) { res.d[0] = key; res.id[0] = sid; }
        if (len > L) flag = 1;  // more seeds than L: host path
    }

    // ---- lock-step iterations of this query (disk_provider.rs:545-652) ----
    while (!flag) {
        steps++;
        const float thr = len >= L ? res.get_d(L - 1) : __builtin_inff();
        uint64_t best = ~0ull;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int e = s * 64 + lane;
            if (e < len && !(res.id[s] & kExpanded)) {
                const uint64_t c = ((uint64_t)ford(res.d[s]) << 32) | res.id[s];
                best = c < best ? c : best;
            }
        }
        if (nspill) {
            // spill entries above the threshold can only be a stopping pop: drop them (compact)
            const bool keep = lane < nspill && funord((unsigned)(spill >> 32)) <= thr;
            uint64_t km = __ballot(keep);
            if (__popcll(km) != nspill) {
                uint64_t nv = ~0ull;
                int idx = 0;
                while (km) {
                    const int i = __ffsll((unsigned long long)km) - 1;
                    km &= km - 1;
                    const uint64_t v = rl_u64(spill, i);
                    if (lane == idx) nv = v;
                    idx++;
                }
                spill = nv;
                nspill = idx;
            }
            if (lane < nspill) best = spill < best ? spill : best;
        }
        best = wmin_u64(best);
        if (best == ~0ull) break;  // heap empty (or only entries the stop rule rejects)
        const unsigned cid = (unsigned)best;
        const float cd = funord((unsigned)(best >> 32));
        if (len >= L && cd > thr) break;
        // pop: mark expanded, or take it out of the spill list
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s * 64 + lane < len && res.id[s] == cid) res.id[s] |= kExpanded;
        {
            const uint64_t sm = __ballot(lane < nspill && spill == best);
            if (sm) {
                const int at = __ffsll((unsigned long long)sm) - 1;
                const uint64_t lastv = rl_u64(spill, nspill - 1);
                if (lane == at) spill = lastv;
                if (lane == nspill - 1) spill = ~0ull;
                nspill--;
            }
        }
        // expand: neighbours up to the first sentinel, ids < N, visited insert in order
        const uint32_t nb = lane < R ? adj[(size_t)cid * R + lane] : kNone;
        const uint64_t sent = __ballot(lane < R && nb == kNone);
        const int first = sent ? __ffsll((unsigned long long)sent) - 1 : R;
        const bool valid = lane < first && nb < N;
        bool dup = false;
        uint64_t vm = __ballot(valid);
        while (vm) {
            const int i = __ffsll((unsigned long long)vm) - 1;
            vm &= vm - 1;
            if (valid && lane > i && nb == rl_u(nb, i)) dup = true;
        }
        bool fresh = false;
        if (valid && !dup) {
            const unsigned bit = 1u << (nb & 31);
            fresh = !(atomicOr(vis + (nb >> 5), bit) & bit);
        }
        const uint64_t m = __ballot(fresh);
        if (!m) continue;
        evals += __popcll(m);
        const float dd = dists(m, nb);
        // insert_result in neighbour order
        uint64_t mm = m;
        while (mm) {
            const int j = __ffsll((unsigned long long)mm) - 1;
            mm &= mm - 1;
            const float dj = rl_f(dd, j);
            const unsigned idj = rl_u(nb, j);
            if (!(len < L || dj < res.get_d(len - 1))) continue;
            const int pos = res.rust_pos(dj, len);
            float evd = 0.f;
            unsigned evi = kNone;
            if (len == L) { evd = res.get_d(L - 1); evi = res.get_id(L - 1); }
            res.insert_at(pos, dj, idj, lane);
            len++;
            if (len > L) {
                len = L;
                res.clear_at(L, lane);
                // an unexpanded entry evicted on a tie with the new threshold stays poppable
                if (!(evi & kExpanded) && evd == res.get_d(L - 1)) {
                    if (nspill < 64) {
                        if (lane == nspill) spill = ((uint64_t)ford(evd) << 32) | evi;
                        nspill++;
                    } else {
                        flag = 1;
                    }
                }
            }
        }
    }

    // ---- first k of the result (ffi.rs:759-762 padding) ----
    for (int e0 = 0; e0 < k; e0 += 64) {
        const int e = e0 + lane;
        float dv = FLT_MAX;
        int64_t iv = -1;
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s * 64 + lane == e && e < len) { dv = res.d[s]; iv = (int64_t)(res.id[s] & ~kExpanded); }
        if (e < k) {
            out_d[(int64_t)qi * k + e] = dv;
            out_ids[(int64_t)qi * k + e] = iv;
        }
    }
    if (lane == 0) {
        flags[qi] = flag;
        atomicAdd(stats + 0, evals);
        atomicMax(stats + 1, (unsigned long long)steps);
        atomicAdd(stats + 2, (unsigned long long)steps);
    }
}

}  // namespace

// S: result slots per lane (L ≤ 64·S); T: 16-byte chunks per lane (d ≤ 64·T·dims-per-chunk)
bool diskann_bfs_supported(int d, int fmt, int R, int n_ep, int L, uint32_t N) {
    const int dc = fmt == 1 ? 16 : 4;
    return d > 0 && d % dc == 0 && d <= 64 * dc * (fmt == 1 ? 2 : 8) && R > 0 && R <= 64 && n_ep >= 0 &&
           n_ep <= 64 && L >= 1 && L <= 256 && N <= 0x7fffffffu;
}

void launch_diskann_bfs(const float *Q, int nq, int d, int fmt, const void *data, const float2 *ab,
                        const uint32_t *adj, int R, uint32_t N, const uint32_t *eps, int n_ep, int k, int L,
                        int metric, uint32_t *visited, int64_t vwords, int64_t *out_ids, float *out_d, int *flags,
                        unsigned long long *stats, hipStream_t st) {
    if (nq <= 0) return;
    const int dc = fmt == 1 ? 16 : 4;
    const int chunks = (d / dc + 63) / 64;  // 16-B chunks per lane
    const int T = chunks <= 1 ? 1 : chunks <= 2 ? 2 : chunks <= 4 ? 4 : 8;
    const bool s2 = L <= 128;
    const uint8_t *x = static_cast<const uint8_t *>(data);
    dim3 grid((unsigned)nq), block(64);
#define HIPANN_BFS(S_, T_, SQ_, IP_)                                                                           \
    hipLaunchKernelGGL((diskann_bfs<S_, T_, SQ_, IP_>), grid, block, 0, st, Q, nq, d, x, ab, adj, R, N, eps, n_ep, \
                       k, L, visited, vwords, out_ids, out_d, flags, stats)
#define HIPANN_BFS_S(T_, SQ_, IP_) \
    do { if (s2) HIPANN_BFS(2, T_, SQ_, IP_); else HIPANN_BFS(4, T_, SQ_, IP_); } while (0)
#define HIPANN_BFS_M(T_, SQ_) \
    do { if (metric == 1) HIPANN_BFS_S(T_, SQ_, true); else HIPANN_BFS_S(T_, SQ_, false); } while (0)
    if (fmt == 1) {
        if (T == 1) HIPANN_BFS_M(1, true);
        else HIPANN_BFS_M(2, true);
    } else {
        if (T == 1) HIPANN_BFS_M(1, false);
        else if (T == 2) HIPANN_BFS_M(2, false);
        else if (T == 4) HIPANN_BFS_M(4, false);
        else HIPANN_BFS_M(8, false);
    }
#undef HIPANN_BFS_M
#undef HIPANN_BFS_S
#undef HIPANN_BFS
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
