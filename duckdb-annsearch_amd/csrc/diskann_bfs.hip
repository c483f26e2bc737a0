// diskann_bfs.hip — GPU-resident DiskANN beam search (DiskProvider::search_batch on the device).
//
// The reference runs the lock-step best-first search on the host and ships every step's candidate
// vectors to the GPU (rust_lib/src/disk_provider.rs:470-678 → metal_diskann_bridge.mm:255-323): one
// PCIe round trip per step, host hash sets and heaps.  Here the whole traversal of a query runs in
// one workgroup of W = 2 wavefronts with the database (fp32 rows or SQ8 codes), the adjacency (N × R
// u32) and a per-query visited bitmap resident in HBM.  Wave 0 runs the state machine; each step's
// fresh neighbours are split over the W waves for the distance gather (P rows in flight per wave,
// unconditional loads, packed-fp32 arithmetic, one reduce-scatter butterfly for P rows).
//
// Exactness.  Wave 0 reproduces the reference's per-query state machine step for step:
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
#include <type_traits>

namespace hipann {
namespace {

#ifndef HIPANN_BFS_W
#define HIPANN_BFS_W 2  // wavefronts per query (tuning builds: -DHIPANN_BFS_W=1/4)
#endif
#ifndef HIPANN_BFS_PROF
#define HIPANN_BFS_PROF 0  // tuning builds: per-phase shader-clock totals of wave 0 into stats[3..6]
#endif
#ifndef HIPANN_BFS_SPEC
#define HIPANN_BFS_SPEC 0  // speculative row / visited-word fetch of the next expansion (measured slower, off)
#endif
#ifndef HIPANN_BFS_RV
#define HIPANN_BFS_RV 128  // VGPRs of row data in flight per lane (rows_in_flight)
#endif

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr unsigned kNone = 0xffffffffu;
constexpr unsigned kExpanded = 0x80000000u;
#ifndef HIPANN_BFS_BULK
#define HIPANN_BFS_BULK 6  // admitted candidates from which a step merges them at once (65: never)
#endif
constexpr int kBulkMin = HIPANN_BFS_BULK;

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
__device__ __forceinline__ float xshfl(float x, int o);
// wave minimum of a u64: DPP exchanges inside 16-lane rows, ds_bpermute for the last two levels
__device__ __forceinline__ uint64_t wmin_u64(uint64_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned lo = __float_as_uint(xshfl(__uint_as_float((unsigned)v), o));
        const unsigned hi = __float_as_uint(xshfl(__uint_as_float((unsigned)(v >> 32)), o));
        const uint64_t w = ((uint64_t)hi << 32) | lo;
        v = w < v ? w : v;
    }
    return v;
}
// lane i ← lane i − 1 (DPP wave_shr:1; lane 0 keeps its own value and is overwritten by the caller)
__device__ __forceinline__ float up1_f(float v, int) {
    const int x = __float_as_int(v);
    return __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ unsigned up1_u(unsigned v, int) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}

// Row chunks: 8 SQ8 codes (8 B; 1536 codes = 3 chunks per lane exactly) or 4 floats (16 B); lane `l`,
// chunk t covers chunk index l + 64t.
#ifndef HIPANN_BFS_SQ8_CHUNK
#define HIPANN_BFS_SQ8_CHUNK 8  // bytes of SQ8 codes per lane-load (8: global_load_dwordx2, 16: dwordx4)
#endif
template <bool SQ8> struct Fmt;
template <> struct Fmt<true> {
    static constexpr int kDims = HIPANN_BFS_SQ8_CHUNK;
    using Chunk = typename std::conditional<HIPANN_BFS_SQ8_CHUNK == 16, uint4, uint2>::type;
};
template <> struct Fmt<false> {
    static constexpr int kDims = 4;
    using Chunk = uint4;
};
// Rows in flight per wave for a row of `vg` VGPRs per lane: the largest power of two ≤ 32 within a
// budget of HIPANN_BFS_RV VGPRs of row data.
constexpr int rows_in_flight(int vg) {
    int p = 1;
    while (p < 32 && 2 * p * vg <= HIPANN_BFS_RV) p *= 2;
    return p;
}
// Groups of pg rows in flight at once: HIPANN_BFS_RVG VGPRs of row data (0: one group).  At
// 1M × 1536 SQ8 a step has ≈46 fresh neighbours, 23 per wave: 3 groups of 8 (144 VGPRs) load them in
// one round where one group of 16 needed two.
#ifndef HIPANN_BFS_RVG
#define HIPANN_BFS_RVG 0
#endif
constexpr int groups_in_flight(int vg, int pg) {
    int g = 1;
    while ((g + 1) * pg * vg <= HIPANN_BFS_RVG) ++g;
    return g;
}

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
    // slice::binary_search_by(|p| p.0.partial_cmp(&dist).unwrap_or(Equal)).unwrap_or_else(|e| e).
    // With no element equal to dist and no NaN on either side the answer is the unique insertion
    // point, the count of elements < dist (two ballots); otherwise Rust's probe sequence decides
    // which of the equal elements it lands on, replayed exactly by rust_pos_probe.
    __device__ __forceinline__ int rust_pos(float dist, int len, int lane) const {
        int lt = 0;
        bool special = dist != dist;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const bool in = s * 64 + lane < len;
            lt += __popcll(__ballot(in && d[s] < dist));
            special |= __ballot(in && (d[s] == dist || d[s] != d[s])) != 0;
        }
        return special ? rust_pos_probe(dist, len) : lt;
    }
    __device__ __forceinline__ int rust_pos_probe(float dist, int len) const {
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

// Cross-lane xor exchange: DPP inside a 16-lane row (offsets 1, 2, 4, 8), ds_bpermute beyond.
// `o` is a compile-time constant after unrolling, so only one branch survives.
__device__ __forceinline__ float xshfl(float x, int o) {
    const int v = __float_as_int(x);
    int r;
    if (o == 1) r = __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false);        // quad_perm [1,0,3,2]
    else if (o == 2) r = __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    else if (o == 4) {                                                                // (m ^ 7) ^ 3
        const int h = __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false);
        r = __builtin_amdgcn_update_dpp(h, h, 0x1B, 0xF, 0xF, false);
    } else if (o == 8) r = __builtin_amdgcn_update_dpp(v, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    else return __shfl_xor(x, o);
    return __int_as_float(r);
}

// Sum over the 64 lanes of P per-lane partials at once (reduce-scatter butterfly): step s halves the
// live values by exchanging with lane ^ (32 >> s), so P rows cost P − 1 + 6 − log2 P exchanges instead
// of 6·P.  On return, lanes [64/P·r, 64/P·(r+1)) hold the total of row r.
template <int P>
__device__ __forceinline__ float reduce_rows(float (&v)[P], int lane) {
    constexpr int LP = P >= 64 ? 6 : P >= 32 ? 5 : P >= 16 ? 4 : P >= 8 ? 3 : P >= 4 ? 2 : P >= 2 ? 1 : 0;
    static_assert((1 << LP) == P, "P must be a power of two <= 64");
#pragma unroll
    for (int s = 0; s < LP; ++s) {
        const int o = 32 >> s, half = P >> (s + 1);
        const int bm = (lane & o) ? -1 : 0;  // bit-mask selects: a `b ? v[i] : v[i + half]` becomes a
#pragma unroll                               // dynamically indexed (scratch) array in hipcc
        for (int i = 0; i < half; ++i) {
            const int lo = __float_as_int(v[i]), hi = __float_as_int(v[i + half]);
            const float send = __int_as_float((lo & bm) | (hi & ~bm));
            const float keep = __int_as_float((hi & bm) | (lo & ~bm));
            v[i] = keep + xshfl(send, o);
        }
    }
    float x = v[0];
#pragma unroll
    for (int o = 32 >> LP; o >= 1; o >>= 1) x += xshfl(x, o);
    return x;
}

// One block of W wavefronts per query.  Wave 0 owns the search state (result list, spill list, stop
// rule) and does the expansions; a step's fresh neighbours go to all W waves through LDS, each wave
// loads its share of the rows with P rows in flight, and the distances come back through LDS for
// wave 0's inserts (two barriers per step; steps without fresh neighbours stay inside wave 0).
template <int S, int T, int W, bool SQ8, bool IP>
__global__ void __launch_bounds__(64 * W)
diskann_bfs(const float *__restrict__ Qs, int nq, int d, const uint8_t *__restrict__ data,
            const float2 *__restrict__ ab, const uint32_t *__restrict__ adj, const uint32_t *__restrict__ dupw,
            int R, uint32_t N, const uint32_t *__restrict__ eps, int n_ep, int k, int L, uint32_t *__restrict__ visited,
            int64_t vwords, int64_t *__restrict__ out_ids, float *__restrict__ out_d, int *__restrict__ flags,
            unsigned long long *__restrict__ stats) {
    constexpr int DC = Fmt<SQ8>::kDims;
    using Chunk = typename Fmt<SQ8>::Chunk;
    constexpr int CB = (int)sizeof(Chunk);
    // rows in flight per wave: P = NG groups of PG (a power of two, one reduce-scatter per group)
    constexpr int PG = rows_in_flight(T * CB / 4);
    constexpr int NG = groups_in_flight(T * CB / 4, PG);
    constexpr int P = PG * NG;
    constexpr int LP = PG >= 32 ? 5 : PG >= 16 ? 4 : PG >= 8 ? 3 : PG >= 4 ? 2 : PG >= 2 ? 1 : 0;
    __shared__ uint32_t s_ids[64];  // this step's fresh neighbours, in neighbour order
    __shared__ float s_dist[64];    // their distances
    __shared__ int s_cnt;           // how many; −1 = the query is done
    __shared__ __attribute__((aligned(16))) uint32_t s_nb[64];  // wave 0: the expansion's neighbour ids
    // wave 0, bulk insert: the result list, the sorted admitted candidates, the merged list
    __shared__ float s_ld[64 * S], s_md[64 * S], s_cd[64];
    __shared__ uint32_t s_mi[64 * S];
    const int qi = blockIdx.x;
    if (qi >= nq) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const size_t rowbytes = SQ8 ? (size_t)d : (size_t)d * 4;
    uint32_t *vis = visited + (int64_t)qi * vwords;
    const float *q = Qs + (int64_t)qi * d;

    // per-lane query terms for the lane's dims (chunk t: dims DC·(lane + 64t) ..), as pairs for the
    // packed-fp32 VALU (v_pk_fma_f32: two lanes of arithmetic per instruction)
    f32x2 qp[T][DC / 2], av[T][DC / 2];
    float cq = 0.f;
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int e = 0; e < DC; ++e) {
            const int dim = DC * (lane + 64 * t) + e;
            // unconditional (clamped) loads: a branch per element serialises them on vmcnt(0)
            const bool in = dim < d;
            const int dc = in ? dim : 0;
            float qv = in ? q[dc] : 0.f, a = 0.f, b = 0.f;
            if (SQ8) {
                const float2 p = ab[dc];
                a = in ? p.x : 0.f;
                b = in ? p.y : 0.f;
            }
            float x, y;
            if (SQ8) {
                if (IP) { x = qv * a; cq = fmaf(qv, b, cq); }
                else { x = qv - b; }
                y = a;
            } else {
                x = qv;
                y = 0.f;
            }
            qp[t][e >> 1][e & 1] = x;
            av[t][e >> 1][e & 1] = y;
        }
    if (SQ8 && IP) cq = wsum(cq);

    auto load_row = [&](uint32_t rid, Chunk (&v)[T]) {
        const uint8_t *base = data + (size_t)rid * rowbytes;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            // unconditional loads (a load under a branch costs a vmcnt(0) per row): past the row's
            // end a lane re-reads the row's first chunk and the value is zeroed afterwards
            const size_t off = (size_t)CB * (lane + 64 * t);
            const bool in = off < rowbytes;
            const Chunk c = *reinterpret_cast<const Chunk *>(base + (in ? off : 0));
            v[t] = in ? c : Chunk{};
        }
    };
    // this lane's partial of one row's distance (the cross-lane sum is reduce_rows)
    auto row_part = [&](const Chunk (&v)[T]) -> float {
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int t = 0; t < T; ++t) {
            if constexpr (SQ8) {
                unsigned w[4];
                __builtin_memcpy(w, &v[t], sizeof(Chunk));
#pragma unroll
                for (int e = 0; e < DC / 2; ++e) {
                    const unsigned ww = w[e >> 1] >> (16 * (e & 1));
                    const f32x2 c = {(float)(ww & 0xffu), (float)((ww >> 8) & 0xffu)};
                    if (IP) acc = __builtin_elementwise_fma(qp[t][e], c, acc);
                    else {
                        const f32x2 tt = __builtin_elementwise_fma(-c, av[t][e], qp[t][e]);
                        acc = __builtin_elementwise_fma(tt, tt, acc);
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const f32x2 x = {__uint_as_float(e ? v[t].z : v[t].x), __uint_as_float(e ? v[t].w : v[t].y)};
                    if (IP) acc = __builtin_elementwise_fma(qp[t][e], x, acc);
                    else {
                        const f32x2 tt = qp[t][e] - x;
                        acc = __builtin_elementwise_fma(tt, tt, acc);
                    }
                }
            }
        }
        return acc[0] + acc[1];
    };
    // Distances of the step's fresh rows s_ids[0, cnt) into s_dist: wave w takes a contiguous share,
    // P rows in flight at a time (rows past the share re-load its last row; their sums are dropped).
    // Distances of the step's fresh rows s_ids[0, cnt) into s_dist: wave w takes a contiguous share,
    // P rows in flight at a time (rows past the share re-load its last row; their sums are dropped).
    // (Pipelining the next round's loads behind this round's arithmetic needs P = 8 to fit 2 waves
    // per SIMD, and measured 2.62 ms against 2.54 ms for two P = 16 rounds.)
    auto dist_phase = [&](int cnt) {
        const int per = (cnt + W - 1) / W;
        const int r_begin = wave * per;
        const int r_end = cnt < r_begin + per ? cnt : r_begin + per;
        for (int r0 = r_begin; r0 < r_end; r0 += P) {
            Chunk v[P][T];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int r = r0 + p < r_end ? r0 + p : r_end - 1;
                load_row((uint32_t)__builtin_amdgcn_readfirstlane((int)s_ids[r]), v[p]);
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if (NG > 1 && r0 + g * PG >= r_end) break;  // wave-uniform
                float part[PG];
#pragma unroll
                for (int p = 0; p < PG; ++p) part[p] = row_part(v[g * PG + p]);
                const float tot = reduce_rows<PG>(part, lane);
                const int r = r0 + g * PG + (lane >> (6 - LP));
                if ((lane & ((64 >> LP) - 1)) == 0 && r < r_end) s_dist[r] = IP ? -(tot + cq) : tot;
            }
        }
    };

    ResultList<S> res;
#pragma unroll
    for (int s = 0; s < S; ++s) { res.d[s] = __builtin_inff(); res.id[s] = kNone; }
    int len = 0;

    // Bulk insert (wave 0): returns false, with the list untouched, when any admitted distance is
    // non-finite or equals another admitted or listed distance, or two listed distances are equal —
    // the sequential Rust-order inserts then run as before.
    auto bulk_insert = [&](uint64_t am, float dd, unsigned nbr) -> bool {
        const bool adm = (am >> lane) & 1ull;
        const int nA = __popcll(am);
        if (__ballot(adm && !(__builtin_fabsf(dd) < __builtin_inff()))) return false;
        // admitted candidates sorted ascending (ties only among the non-admitted +inf keys)
        float key = adm ? dd : __builtin_inff();
        int src = lane;
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const float ok2 = __shfl_xor(key, stride);
                const int os = __shfl_xor(src, stride);
                const bool keep_min = ((lane & stride) == 0) == ((lane & size) == 0);
                const bool o_less = ok2 < key || (ok2 == key && os < src);
                if (keep_min == o_less) { key = ok2; src = os; }
            }
        const unsigned cid = (unsigned)__shfl((int)nbr, src);
        __builtin_amdgcn_wave_barrier();
        s_cd[lane] = key;
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s * 64 + lane < len) s_ld[s * 64 + lane] = res.d[s];
        __builtin_amdgcn_wave_barrier();
        bool bad = lane + 1 < nA && s_cd[lane + 1] == key;  // equal admitted distances
        // list elements: new position e + #(candidates < d_e); a candidate equal to d_e is a tie
        int np_l[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int e = s * 64 + lane;
            const float de = res.d[s];
            int c = 0;
#pragma unroll
            for (int b = 64; b > 0; b >>= 1)
                if (c + b <= nA && s_cd[c + b - 1] < de) c += b;
            np_l[s] = e + c;
            if (e < len) bad |= (c < nA && s_cd[c] == de) || !(de == de) || (e + 1 < len && s_ld[e + 1] == de);
        }
        // candidates: new position i + #(list elements < key)
        int cl = 0;
#pragma unroll
        for (int b = 128 * (S > 2 ? 2 : 1); b > 0; b >>= 1)
            if (cl + b <= len && s_ld[cl + b - 1] < key) cl += b;
        const int np_c = lane + cl;
        if (__ballot(bad)) return false;
        const int nlen = len + nA < L ? len + nA : L;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (s * 64 + lane < len && np_l[s] < nlen) { s_md[np_l[s]] = res.d[s]; s_mi[np_l[s]] = res.id[s]; }
        if (lane < nA && np_c < nlen) { s_md[np_c] = key; s_mi[np_c] = cid; }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int e = s * 64 + lane;
            res.d[s] = e < nlen ? s_md[e] : __builtin_inff();
            res.id[s] = e < nlen ? s_mi[e] : kNone;
        }
        len = nlen;
        return true;
    };
    uint64_t spill = ~0ull;  // lane < nspill: a heap entry evicted from result on a boundary tie
    int nspill = 0;
    int flag = 0;
    unsigned long long evals = 0;
    int steps = 0;
    // Speculated next expansion (wave 0).  The adjacency row and the visited words of the entry most
    // likely to be popped next are fetched while the current step's rows are gathered or inserted, so a
    // correct guess starts the next step's gather without the two dependent round trips (adjacency,
    // then visited).  A guess never changes what is computed: it is used only when its id equals the
    // popped one, its visited words were read after every mark of earlier steps (only this workgroup
    // writes this bitmap), and each mark it implies is confirmed by the returned old word (a
    // mismatch flags the query for the host path).
    //   sp_state 0: nothing; 1: sp_nb / sp_md loaded; 2: sp_w (visited word of lane's neighbour) too.
    unsigned sp_id = kNone;
    uint32_t sp_nb = kNone, sp_w = 0;
    bool sp_md = true;
    int sp_state = 0;
    unsigned long long sp_hits = 0;
    uint64_t mark_lanes = 0;    // this step's speculative marks: lanes whose old word must be unmarked
    uint32_t mark_old = 0, mark_bit = 0;
    auto adj_row = [&](unsigned id, uint32_t &nb_out, bool &md_out) {
        nb_out = lane < R ? adj[(size_t)id * R + lane] : kNone;
        md_out = dupw == nullptr || ((dupw[id >> 5] >> (id & 31)) & 1u);
    };
    // visited words of a row's valid neighbours: device-scope loads, which bypass the CU's L1 and read
    // L2, where the marks (atomics) land
    auto visited_words = [&](uint32_t nbv) -> uint32_t {
        const uint64_t s = __ballot(lane < R && nbv == kNone);
        const int f = s ? __ffsll((unsigned long long)s) - 1 : R;
        return (lane < f && nbv < N) ? __hip_atomic_load(vis + (nbv >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0u;
    };

    const uint64_t lanes_below = (1ull << lane) - 1;  // lane 63: all lower lanes (no overflow)
#if HIPANN_BFS_PROF
    unsigned long long tprof[6] = {0, 0, 0, 0, 0, 0};
    long long tmark = clock64();
#define BFS_T(i)                            \
    do {                                    \
        const long long t1_ = clock64();    \
        tprof[i] += (unsigned long long)(t1_ - tmark); \
        tmark = t1_;                        \
    } while (0)
#else
#define BFS_T(i) \
    do {         \
    } while (0)
#endif

    // ---- seeds (disk_provider.rs:524-538): visited insert in order, distance, push, stable sort ----
    if (wave == 0) {
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
        if (fresh) s_ids[__popcll(m & lanes_below)] = ep;
        if (lane == 0) s_cnt = __popcll(m);
    }
    __syncthreads();
    if (s_cnt > 0) dist_phase(s_cnt);
    __syncthreads();
    if (wave == 0) {
        // stable sort by distance: key (dist, rank) lexicographic (rank = seed order); non-seeds last
        const int c = s_cnt;
        float key = lane < c ? s_dist[lane] : __builtin_inff();
        int src = lane < c ? lane : 64 + lane;
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
        len = c;
        const uint32_t sid = s_ids[src & 63];
        if (lane < len) { res.d[0] = key; res.id[0] = sid; }
        if (len > L) flag = 1;  // more seeds than L: host path
    }

    // ---- lock-step iterations of this query (disk_provider.rs:545-652) ----
    for (;;) {
      int cnt = -1;  // fresh neighbours of this step's expansion (−1: the query is done)
      if (wave == 0) {
        while (!flag) {
        steps++;
        if (sp_state == 1) {  // a guessed row arrived during the inserts: its visited words now
            sp_w = visited_words(sp_nb);
            sp_state = 2;
        }
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
        BFS_T(0);
        // expand: neighbours up to the first sentinel, ids < N, visited insert in order
        const bool hit = HIPANN_BFS_SPEC && sp_state != 0 && cid == sp_id;
        const bool hit_w = hit && sp_state == 2;
        sp_hits += hit ? 1 : 0;
        uint32_t nb;
        // rows flagged at registration as holding a repeated id before their first sentinel (none in
        // a Vamana graph) take the dedupe below; every other row skips it
        bool maydup;
        if (hit) { nb = sp_nb; maydup = sp_md; }
        else adj_row(cid, nb, maydup);
        sp_state = 0;
        const uint64_t sent = __ballot(lane < R && nb == kNone);
        BFS_T(1);
        const int first = sent ? __ffsll((unsigned long long)sent) - 1 : R;
        const bool valid = lane < first && nb < N;
        bool dup = false;
        if (maydup) {
        // first occurrence wins: compare with every earlier lane's id through LDS broadcast reads
        // (invalid lanes hold 0x80000000 | lane, which no id < N ≤ 2^31 − 1 equals)
        s_nb[lane] = valid ? nb : (0x80000000u | (unsigned)lane);
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int i = 0; i < 64; i += 4) {  // 4 broadcast reads in flight per iteration (lanes ≥ first hold sentinels)
            const uint4 w = *reinterpret_cast<const uint4 *>(s_nb + i);
            dup |= (i < lane && w.x == nb) | (i + 1 < lane && w.y == nb) | (i + 2 < lane && w.z == nb) |
                   (i + 3 < lane && w.w == nb);
        }
        dup = dup && valid;
        __builtin_amdgcn_wave_barrier();
        }
        BFS_T(2);
        bool fresh = false;
        const unsigned bit = 1u << (nb & 31);
        mark_lanes = 0;
        if (hit_w) {
            // visited words read after every earlier mark: fresh is decided now; the marks go out
            // and their old words are checked after the gather
            fresh = valid && !dup && !(sp_w & bit);
            if (fresh) mark_old = atomicOr(vis + (nb >> 5), bit);
            mark_bit = bit;
            mark_lanes = __ballot(fresh);
        } else if (valid && !dup) {
            fresh = !(atomicOr(vis + (nb >> 5), bit) & bit);
        }
        const uint64_t m = __ballot(fresh);
        BFS_T(3);
        if (!m) continue;
        evals += __popcll(m);
        if (fresh) s_ids[__popcll(m & lanes_below)] = nb;  // neighbour order
        cnt = __popcll(m);
        break;
        }  // while (!flag)
        if (lane == 0) s_cnt = cnt;
      }  // wave 0
      __syncthreads();
      cnt = s_cnt;
      if (cnt < 0) break;
      dist_phase(cnt);
      __syncthreads();
      if (wave == 0) {
        BFS_T(4);
        // the speculative marks' old words: each must have been unmarked, as the guess assumed
        if (__ballot(((mark_lanes >> lane) & 1ull) && (mark_old & mark_bit))) flag = 1;
        mark_lanes = 0;
        // insert_result in neighbour order
        const float dd = lane < cnt ? s_dist[lane] : 0.f;
        const unsigned nbr = lane < cnt ? s_ids[lane] : kNone;
        // The threshold result[L−1] only falls once the list is full, so a candidate at or above the
        // step's starting threshold is rejected whenever its turn comes: visit only the others.
        const bool full = len >= L;
        const float thr0 = full ? res.get_d(len - 1) : 0.f;
        uint64_t am = __ballot(lane < cnt && (!full || dd < thr0));
        if (HIPANN_BFS_SPEC) {
            // the next pop is almost always the smallest of the unexpanded entries, the spill list and the
            // admitted candidates (a superset of what the inserts leave poppable): fetch its adjacency row
            // behind the inserts; its visited words go out at the top of the next step
            uint64_t b = ~0ull;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int e = s * 64 + lane;
                if (e < len && !(res.id[s] & kExpanded)) {
                    const uint64_t c = ((uint64_t)ford(res.d[s]) << 32) | res.id[s];
                    b = c < b ? c : b;
                }
            }
            if (lane < nspill) b = spill < b ? spill : b;
            if ((am >> lane) & 1ull) {
                const uint64_t c = ((uint64_t)ford(dd) << 32) | nbr;
                b = c < b ? c : b;
            }
            b = wmin_u64(b);
            if (b != ~0ull) {
                sp_id = (unsigned)b;
                adj_row(sp_id, sp_nb, sp_md);
                sp_state = 1;
            }
        }
        // Many admitted candidates and no equal / non-finite distance anywhere: the inserts in neighbour
        // order end in exactly the first L of the sorted union (each binary search lands on the unique
        // insertion point; a candidate rejected at its turn already had L smaller entries ahead of it;
        // with no equal values no eviction is a boundary tie, so nothing spills) — one merge instead.
        if (__popcll(am) >= kBulkMin && bulk_insert(am, dd, nbr)) am = 0;
        while (am) {
            const int j = __ffsll((unsigned long long)am) - 1;
            am &= am - 1;
            const float dj = rl_f(dd, j);
            const unsigned idj = rl_u(nbr, j);
            if (!(len < L || dj < res.get_d(len - 1))) continue;
            const int pos = res.rust_pos(dj, len, lane);
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
        BFS_T(5);
      }
    }
    if (wave != 0) return;
#if HIPANN_BFS_PROF
    if (lane == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(stats + 3 + i, tprof[i]);
#endif
#undef BFS_T

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
        atomicAdd(stats + 9, sp_hits);
    }
}

// dupw bit r = adjacency row r holds some id twice before its first u32::MAX (one wave per row)
__global__ void __launch_bounds__(256) diskann_dup_rows(const uint32_t *__restrict__ adj, int R, int64_t n,
                                                        uint32_t *__restrict__ dupw) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const uint32_t v = lane < R ? adj[row * R + lane] : kNone;
    const uint64_t sent = __ballot(lane < R && v == kNone);
    const int first = sent ? __ffsll((unsigned long long)sent) - 1 : R;
    bool dup = false;
    for (int i = 0; i < first; ++i) dup |= lane > i && lane < first && v == rl_u(v, i);
    if (__ballot(dup) && lane == 0) atomicOr(dupw + (row >> 5), 1u << (row & 31));
}

}  // namespace

void launch_diskann_dup_rows(const uint32_t *adj, int R, int64_t n, uint32_t *dupw, hipStream_t st) {
    HIPANN_CHECK(hipMemsetAsync(dupw, 0, (size_t)((n + 31) / 32) * 4, st));
    if (n <= 0) return;
    HIPANN_REQUIRE(R > 0 && R <= 64 && (n + 3) / 4 < (int64_t)0x7fffffff, "diskann_dup_rows: bad shape");
    hipLaunchKernelGGL(diskann_dup_rows, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, adj, R, n, dupw);
    HIPANN_CHECK(hipGetLastError());
}

// S: result slots per lane (L ≤ 64·S); T: row chunks per lane (8 codes or 4 floats each)
bool diskann_bfs_supported(int d, int fmt, int R, int n_ep, int L, uint32_t N) {
    const int dc = fmt == 1 ? HIPANN_BFS_SQ8_CHUNK : 4;
    return d > 0 && d % dc == 0 && d <= 64 * dc * (fmt == 1 ? 4 : 8) && R > 0 && R <= 64 && n_ep >= 0 &&
           n_ep <= 64 && L >= 1 && L <= 256 && N <= 0x7fffffffu;
}

void launch_diskann_bfs(const float *Q, int nq, int d, int fmt, const void *data, const float2 *ab,
                        const uint32_t *adj, const uint32_t *dupw, int R, uint32_t N, const uint32_t *eps, int n_ep, int k, int L,
                        int metric, uint32_t *visited, int64_t vwords, int64_t *out_ids, float *out_d, int *flags,
                        unsigned long long *stats, hipStream_t st) {
    if (nq <= 0) return;
    HIPANN_REQUIRE(diskann_bfs_supported(d, fmt, R, n_ep, L, N), "diskann_bfs: unsupported shape");
    const int dc = fmt == 1 ? HIPANN_BFS_SQ8_CHUNK : 4;
    const int chunks = (d / dc + 63) / 64;  // row chunks per lane
    const bool s2 = L <= 128;
    const uint8_t *x = static_cast<const uint8_t *>(data);
    constexpr int W = HIPANN_BFS_W;
    dim3 grid((unsigned)nq), block(64 * W);
#define HIPANN_BFS(S_, T_, SQ_, IP_)                                                                              \
    hipLaunchKernelGGL((diskann_bfs<S_, T_, W, SQ_, IP_>), grid, block, 0, st, Q, nq, d, x, ab, adj, dupw, R, N, eps, n_ep, \
                       k, L, visited, vwords, out_ids, out_d, flags, stats)
#define HIPANN_BFS_S(T_, SQ_, IP_) \
    do { if (s2) HIPANN_BFS(2, T_, SQ_, IP_); else HIPANN_BFS(4, T_, SQ_, IP_); } while (0)
#define HIPANN_BFS_M(T_, SQ_) \
    do { if (metric == 1) HIPANN_BFS_S(T_, SQ_, true); else HIPANN_BFS_S(T_, SQ_, false); } while (0)
    if (fmt == 1) {
        if (chunks <= 1) HIPANN_BFS_M(1, true);
        else if (chunks <= 2) HIPANN_BFS_M(2, true);
        else if (chunks <= 3) HIPANN_BFS_M(3, true);
        else HIPANN_BFS_M(4, true);
    } else {
        if (chunks <= 1) HIPANN_BFS_M(1, false);
        else if (chunks <= 2) HIPANN_BFS_M(2, false);
        else if (chunks <= 4) HIPANN_BFS_M(4, false);
        else if (chunks <= 6) HIPANN_BFS_M(6, false);
        else HIPANN_BFS_M(8, false);
    }
#undef HIPANN_BFS_M
#undef HIPANN_BFS_S
#undef HIPANN_BFS
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
