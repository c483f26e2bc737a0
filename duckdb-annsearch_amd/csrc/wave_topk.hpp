// wave_topk.hpp — wave64-distributed sorted top-k lists for CDNA4 (gfx950).
//
// A list of up to 64*S (key, id) pairs lives in S registers pairs of ONE wavefront: element
// e = s*64 + lane sits in slot s of lane `lane`.  The list is kept sorted ascending by the
// lexicographic order (key, id).  Selecting the k smallest pairs of a candidate stream by that
// order is exactly FAISS's result: its heaps admit a candidate only when it is strictly better than
// the current worst and break equal distances by label (faiss::CMax::cmp2 / heap_reorder), and the
// extension's Metal selects keep "earlier index wins" on ties (warp_select.metal:37-58).  Because
// the lexicographic top-k of a multiset does not depend on arrival order, partial lists computed by
// different waves / blocks / GPUs merge exactly.
//
// Insert cost: one ballot + one popcount + one shuffle per slot — no per-lane serial loop.
// Candidates are filtered with a wave-uniform threshold (element k-1) first, so after warm-up
// almost no candidate reaches the insert.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hipann {

constexpr int kWave = 64;
constexpr int kBulkOffer = 12;  // WaveList<1>::offer: more entrants than this → sort + bulk merge

template <typename IdT>
__device__ __forceinline__ bool lex_less(float ad, IdT aid, float bd, IdT bid) {
    return ad < bd || (ad == bd && aid < bid);
}

template <typename IdT> struct IdTraits;
template <> struct IdTraits<int> {
    static __device__ __forceinline__ int pad() { return 0x7fffffff; }
};
template <> struct IdTraits<long long> {
    static __device__ __forceinline__ long long pad() { return 0x7fffffffffffffffLL; }
};

__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ int readlane_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ long long readlane_i(long long v, int lane) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v & 0xffffffffLL), lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)v >> 32), lane);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Shift-up by one lane across the wave (lane 0 receives garbage; callers overwrite it).
__device__ __forceinline__ float shfl_up1_f(float v) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute((int)((lane_id() - 1) & 63) << 2, __float_as_int(v)));
}
__device__ __forceinline__ int shfl_up1_i(int v) {
    return __builtin_amdgcn_ds_bpermute((int)((lane_id() - 1) & 63) << 2, v);
}
__device__ __forceinline__ long long shfl_up1_i(long long v) {
    const int a = (int)((lane_id() - 1) & 63) << 2;
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(a, (int)(unsigned)(v & 0xffffffffLL));
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(a, (int)(unsigned)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// Compare-exchange with lane ^ stride in (key, id) lexicographic order: keep the smaller pair when
// keep_min, else the larger.  Both lanes see the same pair, so the exchange is consistent.
template <typename IdT>
__device__ __forceinline__ void wave_cmpx(float &k, IdT &id, int stride, bool keep_min) {
    const float ok = __shfl_xor(k, stride);
    const IdT oid = __shfl_xor(id, stride);
    const bool take = keep_min ? lex_less(ok, oid, k, id) : lex_less(k, id, ok, oid);
    if (take) { k = ok; id = oid; }
}

// Bitonic sort of one (key, id) per lane, ascending across the wave (21 compare-exchange stages).
template <typename IdT>
__device__ __forceinline__ void wave_sort(float &k, IdT &id) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const bool up = (lane & size) == 0;  // size = 64: every lane ascending
            wave_cmpx(k, id, stride, ((lane & stride) == 0) == up);
        }
}

// Ascending (key, id) order of the first n lanes' pairs (n ≤ 64, wave-uniform; lanes ≥ n end as (+inf, pad)):
// each lane counts the pairs below its own (n broadcasts, no shuffle chain), then one ds_permute per word moves
// every pair to its rank.  Keys compare as order-preserving bits (−0 = +0, NaN last), equal pairs by lane, so the
// ranks are a permutation whatever the input.
template <typename IdT>
__device__ __forceinline__ void wave_rank_sort(float &k, IdT &id, int n) {
    const int lane = threadIdx.x & 63;
    const float kz = k == 0.f ? 0.f : k;
    const unsigned kb = k == k ? ((__float_as_uint(kz) >> 31) ? ~__float_as_uint(kz) : (__float_as_uint(kz) | 0x80000000u))
                               : 0xffffffffu;
    int rank = 0;
    for (int j = 0; j < n; ++j) {
        const unsigned bj = (unsigned)__builtin_amdgcn_readlane((int)kb, j);
        const IdT ij = readlane_i(id, j);
        rank += (bj < kb || (bj == kb && (ij < id || (ij == id && j < lane)))) ? 1 : 0;
    }
    const bool live = lane < n;
    const int dst = (live ? rank : lane) << 2;  // lanes >= n keep their place (their pads stay pads)
    const float kr = __int_as_float(__builtin_amdgcn_ds_permute(dst, __float_as_int(live ? k : __builtin_inff())));
    IdT ir;
    if constexpr (sizeof(IdT) == 8) {
        const unsigned long long u = (unsigned long long)(live ? id : IdTraits<IdT>::pad());
        const unsigned lo = (unsigned)__builtin_amdgcn_ds_permute(dst, (int)(unsigned)(u & 0xffffffffull));
        const unsigned hi = (unsigned)__builtin_amdgcn_ds_permute(dst, (int)(unsigned)(u >> 32));
        ir = (IdT)(((unsigned long long)hi << 32) | lo);
    } else {
        ir = (IdT)__builtin_amdgcn_ds_permute(dst, (int)(live ? id : IdTraits<IdT>::pad()));
    }
    k = lane < n ? kr : __builtin_inff();
    id = lane < n ? ir : IdTraits<IdT>::pad();
}

// One wave-distributed list of 64*S elements.
template <int S, typename IdT = int>
struct WaveList {
    float d[S];
    IdT id[S];

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            d[s] = __builtin_inff();
            id[s] = IdTraits<IdT>::pad();
        }
    }

    // Threshold = element kth (0-based, wave-uniform, kth < 64*S).
    __device__ __forceinline__ void threshold(int kth, float &td, IdT &tid) const {
        const int s = kth >> 6, l = kth & 63;
        float v = d[0];
        IdT vi = id[0];
#pragma unroll
        for (int t = 1; t < S; ++t)
            if (s == t) { v = d[t]; vi = id[t]; }
        td = readlane_f(v, l);
        tid = readlane_i(vi, l);
    }

    // Insert a wave-uniform candidate (cd, cid).  Elements pushed past 64*S are dropped.
    __device__ __forceinline__ void insert(float cd, IdT cid) {
        const int lane = lane_id();
        int pos = 0;
#pragma unroll
        for (int s = 0; s < S; ++s) pos += __popcll(__ballot(lex_less(d[s], id[s], cd, cid)));
#pragma unroll
        for (int s = S - 1; s >= 0; --s) {
            float ud = shfl_up1_f(d[s]);
            IdT uid = shfl_up1_i(id[s]);
            if (s > 0) {
                // lane 0 of slot s receives lane 63 of slot s-1 (still unmodified: we go high→low)
                float cd63 = readlane_f(d[s - 1], 63);
                IdT ci63 = readlane_i(id[s - 1], 63);
                if (lane == 0) { ud = cd63; uid = ci63; }
            }
            const int e = s * 64 + lane;
            if (e == pos) { d[s] = cd; id[s] = cid; }
            else if (e > pos) { d[s] = ud; id[s] = uid; }
        }
    }

    // Offer 64 per-lane candidates (one per lane, any order).  `kth` = k-1.  Candidates whose key is
    // +inf with the padding id never enter.  BULK = false keeps the serial insert only (smaller code,
    // for kernels at a register budget edge).
    template <bool BULK = true>
    __device__ __forceinline__ void offer(float cd, IdT cid, int kth) {
        float td; IdT tid;
        threshold(kth, td, tid);
        bool pass = lex_less(cd, cid, td, tid);
        unsigned long long m = __ballot(pass);
        if constexpr (S == 1 && BULK) {
            // many entrants (an empty list, the first tiles of a scan): one bitonic sort of the
            // passing candidates + a bulk merge instead of one serial insert each
            if (__popcll(m) > kBulkOffer) {
                float ck = pass ? cd : __builtin_inff();
                IdT ci = pass ? cid : IdTraits<IdT>::pad();
                wave_sort(ck, ci);
                merge_sorted(ck, ci);
                return;
            }
        }
        while (m) {
            const int j = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const float xd = readlane_f(cd, j);
            const IdT xi = readlane_i(cid, j);
            // re-check against the current threshold (it tightens as we insert)
            float t2d; IdT t2i;
            threshold(kth, t2d, t2i);
            if (lex_less(xd, xi, t2d, t2i)) insert(xd, xi);
        }
    }

    // Bulk merge (S = 1): (ck, cid) is a wave-sorted ascending run of 64 candidates (wave_sort).
    // min(list, reverse(run)) is bitonic and holds the 64 smallest of the union; six half-cleaner
    // stages sort it.  ≈ 7 shuffle stages, independent of how many candidates enter.
    __device__ __forceinline__ void merge_sorted(float ck, IdT cid) {
        static_assert(S == 1, "bulk merge is for one-slot lists");
        const int lane = lane_id();
        const float rk = __shfl(ck, 63 - lane);
        const IdT rid = __shfl(cid, 63 - lane);
        if (lex_less(rk, rid, d[0], id[0])) { d[0] = rk; id[0] = rid; }
#pragma unroll
        for (int stride = 32; stride > 0; stride >>= 1) wave_cmpx(d[0], id[0], stride, (lane & stride) == 0);
    }

    // Write elements [0, k) to out_d / out_i (lane-strided, coalesced).
    template <typename IdxT>
    __device__ __forceinline__ void store(float *out_d, IdxT *out_i, int k) const {
        const int lane = lane_id();
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int e = s * 64 + lane;
            if (e < k) { out_d[e] = d[s]; out_i[e] = (IdxT)id[s]; }
        }
    }
};

}  // namespace hipann
