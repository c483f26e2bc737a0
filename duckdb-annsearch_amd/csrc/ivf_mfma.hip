// ivf_mfma.hip — IVFFlat list scan on the fp32 matrix cores (gfx950), decomposed form.
//
// Replaces the per-query GEMV-shaped distance + select of MetalIndexIVFFlat::search
// (faiss-metal/src/MetalIndexIVFFlat.mm:122-256, norms stored with the lists at :305-318).  Same
// work plan as the VALU kernels in ivf_kernels.hip (ivf_count / ivf_plan / ivf_fill, slots from
// ivf_slot_scan): an item is (list ℓ, 2048-row chunk of ℓ, group of ≤ G of the queries probing ℓ),
// and every (query, probe, chunk) slot receives exactly one k-list.
//
// The block computes the item's (queries × rows) block of q·x with v_mfma_f32_16x16x4_f32 (exact
// fp32 products, fp32 accumulation: a k-ordered fmaf chain, MI355X_MICROARCH.md §Matrix cores) and
// turns it into  L2: max(0, ‖q‖² + ‖x‖² − 2·q·x)  /  IP: key = −q·x  in registers.
//
// Data movement (the list scan streams each probed list once per batch, so HBM is the roofline):
//   * the item's ≤ G queries are copied once into LDS, all d dims (G = 48 at d = 768: 149 KiB),
//     row stride ≡ 8 dwords (mod 64) so the A-fragment reads (16 queries × one float4) are
//     conflict-free;
//   * rows go straight from HBM into the MFMA B operand: lane (g, m) loads row m's dims
//     16s + 4g .. +3 of a 16-row tile (global_load_dwordx4), P = 6 sixteen-dim steps ahead in a
//     register ring — ≈ 12 KiB in flight per wave, 96 KiB per CU, with no LDS round trip and no
//     barrier in the main loop (cdna_hip_programming.md §5: operand streamed once per block and not
//     shared across waves → load straight to VGPRs, deep unroll).
// Block: 8 waves, one block per CU (LDS).  Wave w takes the item's 32-row passes w, w + 8, … and
// multiplies each pass (2 row tiles) by every query tile (QT ≤ 3): 8·QT MFMAs per 16 dims.
//
// Selection: the accumulator of tile (qt, r) holds, in DPP row g (lanes 16g .. 16g + 15), query
// qt·16 + 4g + v of register v against the tile's 16 rows (lane m = row).  Each wave keeps, per
// query, a sorted list of the k ≤ 16 best (key, row) in one 16-lane DPP row of a register pair — the
// same lanes that hold that query's candidates — so one register pair serves 4 queries and a tile
// merges into the lists with no cross-row traffic: when a 16-row batch has a candidate below a
// lane's cached k-th, the batch is bitonic-sorted inside the rows and merged (reverse + min + 4
// half-cleaner stages), four queries at a time, every exchange a DPP operand.  At the end of the item
// the 8 waves' lists are merged pairwise through LDS (3 rounds) and wave 0 writes the k-lists.
#include "common.hpp"
#include "wave_topk.hpp"

#include <algorithm>
#include <cstdlib>

namespace hipann {

typedef float mf_f32x4 __attribute__((ext_vector_type(4)));

#ifndef HIPANN_MF_EXPERIMENT
#define HIPANN_MF_EXPERIMENT 0  // tuning builds only (wrong results): 1 no selection, 2 no row loads, 3 no MFMA
#endif

#ifndef HIPANN_MF_WAVES
#define HIPANN_MF_WAVES 8
#endif
#ifndef HIPANN_MF_P
#define HIPANN_MF_P 6
#endif
#ifndef HIPANN_MF_QPF
#define HIPANN_MF_QPF 0
#endif
constexpr int MF_WAVES = HIPANN_MF_WAVES;
constexpr int MF_THREADS = 64 * MF_WAVES;
#ifndef HIPANN_IVF_CH
#define HIPANN_IVF_CH 2048
#endif
constexpr int MF_CH = HIPANN_IVF_CH;   // rows per item (= IVF_CH of ivf_kernels.hip)
constexpr int MF_PASS = 32;   // rows per wave pass (2 MFMA row tiles)
constexpr int MF_RT = 2;      // row tiles per pass
constexpr int MF_P = HIPANN_MF_P;  // sixteen-dim steps in flight per wave (register ring depth)
constexpr bool MF_QPF = HIPANN_MF_QPF;  // read the next step's query fragments before this step's MFMAs
constexpr int MF_QTMAX = 3;   // query tiles per item (G ≤ 48)
constexpr int MF_KMAX = 16;   // lists are 16-lane DPP rows
constexpr size_t MF_LDS_MAX = 160 * 1024;

// Dims per query row in LDS (16-dim steps padded to a multiple of the ring depth, zero-filled) and
// the row stride (≡ 8 dwords mod 64: conflict-free ds_read_b128 of 16 rows × one float4).
__host__ __device__ inline int mf_nsub(int d) { return (int)ceil_div(ceil_div(d, 16), MF_P) * MF_P; }
__host__ __device__ inline int mf_stride(int d) { return mf_nsub(d) * 16 + 8; }
inline int mf_group(int d) {
    const int g = (int)(MF_LDS_MAX / ((size_t)mf_stride(d) * 4)) / 16 * 16;
    return g < 16 * MF_QTMAX ? g : 16 * MF_QTMAX;
}

// ---- 16-lane (DPP row) sorted lists ---------------------------------------------------------
// Every exchange partner of the networks below is lane m ^ X inside a 16-lane row, X ∈ {1,2,3,4,7,
// 8,15}: a DPP operand modifier (quad_perm / row_half_mirror / row_mirror / row_ror:8), so a stage
// costs a few VALU ops instead of an LDS-pipe shuffle round trip (ds_bpermute / ds_swizzle latency
// chained through 15 stages made the first version of this epilogue latency-bound).
template <int CTRL>
__device__ __forceinline__ int mf_dpp(int x) {
    return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}
template <int X>
__device__ __forceinline__ int row_xor(int x) {
    if constexpr (X == 1) return mf_dpp<0xB1>(x);              // quad_perm [1,0,3,2]
    else if constexpr (X == 2) return mf_dpp<0x4E>(x);         // quad_perm [2,3,0,1]
    else if constexpr (X == 3) return mf_dpp<0x1B>(x);         // quad_perm [3,2,1,0]
    else if constexpr (X == 7) return mf_dpp<0x141>(x);        // row_half_mirror
    else if constexpr (X == 15) return mf_dpp<0x140>(x);       // row_mirror
    else if constexpr (X == 8) return mf_dpp<0x128>(x);        // row_ror:8
    else { static_assert(X == 4, "row_xor"); return mf_dpp<0x1B>(mf_dpp<0x141>(x)); }  // (m ^ 7) ^ 3
}
template <int X>
__device__ __forceinline__ float row_xor(float x) { return __int_as_float(row_xor<X>(__float_as_int(x))); }

template <int X>
__device__ __forceinline__ uint64_t row_xor(uint64_t x) {
    const unsigned lo = (unsigned)row_xor<X>((int)(unsigned)x), hi = (unsigned)row_xor<X>((int)(unsigned)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// (key, id) packed into one u64 whose unsigned order is the lexicographic (key, id) order: high word
// = the key's order-preserving bits, low word = the shard-local row (pad 0x7fffffff; an empty slot
// is ~0).  One v_cmp_lt_u64 per comparison.
__device__ __forceinline__ unsigned mf_sortable(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float mf_unsortable(unsigned s) {
    return __uint_as_float((s & 0x80000000u) ? (s & 0x7fffffffu) : ~s);
}
constexpr uint64_t MF_EMPTY = ~0ull;
constexpr unsigned MF_PAD_ID = 0x7fffffffu;

// Compare-exchange with lane m ^ X: the lower lane of the pair keeps the smaller, the upper the larger.
template <int X>
__device__ __forceinline__ void row_cx(uint64_t &p, bool upper) {
    const uint64_t o = row_xor<X>(p);
    p = ((o < p) != upper) ? o : p;
}
// Ascending bitonic sort of the 16 packed pairs of every DPP row (mirror form: per block size s a
// mirror stage m ^ (s − 1), then half-cleaners m ^ s/4 … m ^ 1; every stage ascending).
__device__ __forceinline__ void row_sort16(uint64_t &p, int m) {
    row_cx<1>(p, m & 1);
    row_cx<3>(p, m & 2);
    row_cx<1>(p, m & 1);
    row_cx<7>(p, m & 4);
    row_cx<2>(p, m & 2);
    row_cx<1>(p, m & 1);
    row_cx<15>(p, m & 8);
    row_cx<4>(p, m & 4);
    row_cx<2>(p, m & 2);
    row_cx<1>(p, m & 1);
}
// Merge a row-sorted run c into the row-sorted list l: the 16 smallest of the union (min against
// the reversed run is bitonic; four half-cleaner stages sort it).
__device__ __forceinline__ void row_merge16(uint64_t &l, uint64_t c, int m) {
    const uint64_t r = row_xor<15>(c);
    l = r < l ? r : l;
    row_cx<8>(l, m & 8);
    row_cx<4>(l, m & 4);
    row_cx<2>(l, m & 2);
    row_cx<1>(l, m & 1);
}
// Element kth of every row's list, broadcast to the row's lanes (the row's admission threshold).
__device__ __forceinline__ uint64_t row_kth(uint64_t l, int kth, int g) {
    const unsigned lo = (unsigned)l, hi = (unsigned)(l >> 32);
    unsigned rl[4], rh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        rl[r] = (unsigned)__builtin_amdgcn_readlane((int)lo, 16 * r + kth);
        rh[r] = (unsigned)__builtin_amdgcn_readlane((int)hi, 16 * r + kth);
    }
    const unsigned sl = g == 0 ? rl[0] : g == 1 ? rl[1] : g == 2 ? rl[2] : rl[3];
    const unsigned sh = g == 0 ? rh[0] : g == 1 ? rh[1] : g == 2 ? rh[2] : rh[3];
    return ((uint64_t)sh << 32) | sl;
}

// the key word of element kth of every row's list, broadcast to the row's lanes
__device__ __forceinline__ unsigned row_kth_key(uint64_t l, int kth, int g) {
    const unsigned hi = (unsigned)(l >> 32);
    unsigned rh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rh[r] = (unsigned)__builtin_amdgcn_readlane((int)hi, 16 * r + kth);
    return g == 0 ? rh[0] : g == 1 ? rh[1] : g == 2 ? rh[2] : rh[3];
}

// ---- end of an item: the waves' lists → the slot's partial list ------------------------------------
// sub = 0: the 8 waves' lists are merged pairwise through LDS (3 rounds) and wave 0 writes the slot's k-list.
// sub = 1 (the exact forms at request_k > 12, ivf.cpp): no merge — every wave writes its own k-list as
// sub-list `wave` of the slot (MF_WAVES·k entries per slot).  A full sub-list's k-th key still tightens the
// query's running bound, so at the end qbound[q] is the smallest k-th key over the query's full sub-lists:
// every row some sub-list (or the bound) pruned has a scan key ≥ it, which is what ivf_rerank_topk certifies
// against besides its own k-th merged key.
template <int QT>
__device__ __forceinline__ void mf_finish_item(uint64_t (&lst)[QT][4], float *smem, int nqi,
                                               const int *__restrict__ bucket, int boff, int nprobe,
                                               const int *__restrict__ slot_off, int chunk, int k, int sub,
                                               unsigned *__restrict__ qbound, float *__restrict__ part_d,
                                               int *__restrict__ part_i) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = lane & 15, g = lane >> 4;
    if (!sub) {  // block-uniform
        // the query image is dead once every wave has left its main loop (first barrier)
        uint64_t *scratch = reinterpret_cast<uint64_t *>(smem);
#pragma unroll 1
        for (int half = MF_WAVES / 2; half > 0; half >>= 1) {
            __syncthreads();
            if (wave >= half && wave < 2 * half) {
                uint64_t *dst = scratch + (size_t)(wave - half) * QT * 4 * 64;
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int v = 0; v < 4; ++v) dst[(qt * 4 + v) * 64 + lane] = lst[qt][v];
            }
            __syncthreads();
            if (wave < half) {
                const uint64_t *src = scratch + (size_t)wave * QT * 4 * 64;
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int v = 0; v < 4; ++v) row_merge16(lst[qt][v], src[(qt * 4 + v) * 64 + lane], m);
            }
        }
    }
    if ((sub || wave == 0) && m < k) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int q = qt * 16 + 4 * g + v;
                if (q < nqi) {
                    const int pr = bucket[boff + q];
                    const int64_t slot = (int64_t)slot_off[pr] + chunk;
                    const int64_t off = (sub ? slot * MF_WAVES + wave : slot) * k + m;
                    const uint64_t e = lst[qt][v];
                    const unsigned id = (unsigned)e;
                    const bool real = e != MF_EMPTY && id != MF_PAD_ID;
                    part_d[off] = real ? mf_unsortable((unsigned)(e >> 32)) : __builtin_inff();
                    part_i[off] = real ? (int)id : (int)MF_PAD_ID;
                    // a real k-th tightens the query's bound for the items that start later
                    if (m == k - 1 && real) atomicMin(qbound + pr / nprobe, (unsigned)(e >> 32));
                }
            }
    }
}

// ---- one wave's share of an item -----------------------------------------------------------------
template <int QT, bool IP>
__device__ __forceinline__ void mf_item(int d, const float *__restrict__ codes_t, int64_t tp0,
                                        const float *__restrict__ xn,
                                        int64_t r0, int64_t r1, int nqi, const float *__restrict__ qs, int stride,
                                        const float (&qn)[QT][4], const unsigned (&qb)[QT][4],
                                        const int *__restrict__ bucket, int boff, int nprobe,
                                        const int *__restrict__ slot_off, int chunk, int k, int sub, float *smem,
                                        unsigned *__restrict__ qbound, float *__restrict__ part_d,
                                        int *__restrict__ part_i) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = lane & 15, g = lane >> 4;
    const int nsub = mf_nsub(d);               // 16-dim steps per pass (multiple of MF_P)
    const int npass_all = (int)ceil_div(r1 - r0, MF_PASS);
    const int npass = npass_all > wave ? (npass_all - wave + MF_WAVES - 1) / MF_WAVES : 0;  // wave-uniform


    // query validity of the accumulator registers: query qt·16 + 4g + v
    bool qv[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) qv[qt][v] = qt * 16 + 4 * g + v < nqi;

    // Lists start as k copies of (bound, pad): the query's best known k-th key over the items that
    // finished before this one (qbound, any list of this shard), so only rows that can still reach
    // the query's final top-k are ever merged.  Pad entries never reach the output (the merge kernel
    // drops id 0x7fffffff).
    uint64_t lst[QT][4], thr[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint64_t b = ((uint64_t)qb[qt][v] << 32) | MF_PAD_ID;
            lst[qt][v] = m < k ? b : MF_EMPTY;
            thr[qt][v] = b;
        }

    // ---- row stream: step t = (pass i, dim step s).  In the tiled copy a pass's step is 2 KiB
    // contiguous, [row tile r][lane (g, m)][float4]: lane (g, m) of tile r holds row 16r + m, dims
    // 16s + 4g .. +3, so each load is one fully coalesced 1 KiB wave-instruction and a pass streams
    // 96 KiB (d = 768) of consecutive HBM.  The loads are unconditional (past the wave's last step
    // they re-read it): a load under a branch makes hipcc fall back to vmcnt(0) at the loop head.
    auto row_of = [&](int i, int r) -> int64_t {
        const int64_t row = r0 + (int64_t)(wave + MF_WAVES * i) * MF_PASS + 16 * r + m;
        return row < r1 ? row : r1 - 1;
    };
    const int ilast = npass > 0 ? npass - 1 : 0;
    const float *rp;          // this lane's float4 in step 0 of the pass the load stream is in
    int ld_i = 0, ld_s = 0;   // stream position of the next load (wave-uniform)
    auto set_pass = [&](int i) {
        rp = codes_t + ((tp0 + wave + MF_WAVES * i) * nsub) * (MF_RT * 256) + 4 * lane;
    };
    auto next_load = [&](mf_f32x4 (&dst)[MF_RT]) {
        const int s = ld_i <= ilast ? ld_s : nsub - 1;
#pragma unroll
        for (int r = 0; r < MF_RT; ++r)
            dst[r] = *reinterpret_cast<const mf_f32x4 *>(rp + (int64_t)s * (MF_RT * 256) + r * 256);
        if (++ld_s == nsub) {
            ld_s = 0;
            ++ld_i;
            set_pass(ld_i <= ilast ? ld_i : ilast);
        }
    };

    mf_f32x4 ring[MF_P][MF_RT];
    float xnr[MF_RT] = {0.f, 0.f};
    if (npass > 0) {
        set_pass(0);
#pragma unroll
        for (int p = 0; p < MF_P; ++p) next_load(ring[p]);
        if (!IP) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr[r] = xn[row_of(0, r)];
        }
    }

    mf_f32x4 acc[QT][MF_RT];
    uint64_t sink = 0;
    mf_f32x4 qnext[QT];
    if (MF_QPF) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) qnext[qt] = *reinterpret_cast<const mf_f32x4 *>(qs + (qt * 16 + m) * stride + 4 * g);
    }
    for (int i = 0; i < npass; ++i) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) acc[qt][r] = mf_f32x4{0.f, 0.f, 0.f, 0.f};
        float xnr_next[MF_RT] = {0.f, 0.f};
        if (!IP) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr_next[r] = xn[row_of(i + 1 <= ilast ? i + 1 : ilast, r)];
        }
        for (int s0 = 0; s0 < nsub; s0 += MF_P) {
#pragma unroll
            for (int p = 0; p < MF_P; ++p) {
                const int s = s0 + p;
                mf_f32x4 qa[QT];
                if (MF_QPF) {
                    const int sn = s + 1 < nsub ? s + 1 : 0;
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt) {
                        qa[qt] = qnext[qt];
                        qnext[qt] = *reinterpret_cast<const mf_f32x4 *>(qs + (qt * 16 + m) * stride + 16 * sn + 4 * g);
                    }
                } else {
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
                        qa[qt] = *reinterpret_cast<const mf_f32x4 *>(qs + (qt * 16 + m) * stride + 16 * s + 4 * g);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int r = 0; r < MF_RT; ++r)
                            if (HIPANN_MF_EXPERIMENT != 3)
                                acc[qt][r] = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[qt][e], ring[p][r][e], acc[qt][r], 0, 0, 0);
                            else
                                acc[qt][r][e] += qa[qt][e] + ring[p][r][e];
                if (HIPANN_MF_EXPERIMENT != 2) next_load(ring[p]);
            }
        }
        // ---- pass epilogue: keys, filter, merge ----
        const int64_t prow0 = r0 + (int64_t)(wave + MF_WAVES * i) * MF_PASS;
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) {
            const int64_t row = prow0 + 16 * r + m;
            const bool rok = row < r1;
            const unsigned rid = rok ? (unsigned)row : MF_PAD_ID;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    float key;
                    if (IP) {
                        key = -acc[qt][r][v];
                    } else {
                        key = fmaf(-2.f, acc[qt][r][v], qn[qt][v] + xnr[r]);
                        key = key < 0.f ? 0.f : key;
                    }
                    const bool ok = rok && qv[qt][v];
                    key = ok ? key : __builtin_inff();
                    uint64_t cp = ok ? (((uint64_t)mf_sortable(key) << 32) | rid) : MF_EMPTY;
                    if (HIPANN_MF_EXPERIMENT == 1) {
                        sink ^= cp;  // keeps the keys live; the lists (and ids) stay valid
                    } else if (__ballot(cp < thr[qt][v])) {
                        row_sort16(cp, m);
                        row_merge16(lst[qt][v], cp, m);
                        thr[qt][v] = row_kth(lst[qt][v], k - 1, g);
                    }
                }
        }
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) xnr[r] = xnr_next[r];
    }

    if (HIPANN_MF_EXPERIMENT == 1 && sink == 1) part_d[0] = 0.f;

    mf_finish_item<QT>(lst, smem, nqi, bucket, boff, nprobe, slot_off, chunk, k, sub, qbound, part_d, part_i);
}

template <bool IP>
__global__ void __launch_bounds__(MF_THREADS, MF_WAVES / 4)
ivf_scan_mfma(const float *__restrict__ Q, const float *__restrict__ qnorm, int d, const float *__restrict__ codes_t,
              const int64_t *__restrict__ tpass_off,
              const float *__restrict__ xn, const int64_t *__restrict__ list_off, const int *__restrict__ list_len, const int *__restrict__ cnt,
              const int *__restrict__ bucket_off, const int *__restrict__ item_off, const int *__restrict__ bucket,
              const int *__restrict__ slot_off, int nlist, int nprobe, int group, int k, int sub,
              unsigned *__restrict__ qbound, float *__restrict__ part_d, int *__restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int total = item_off[nlist];
    if ((int)blockIdx.x >= total) return;
    const int item = xcd_remap((int)blockIdx.x, total);
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int64_t lr0 = list_off[l], lr1 = lr0 + list_len[l];
    const int c = cnt[l];
    const int ng = (c + group - 1) / group;
    const int rem = item - item_off[l];
    const int chunk = rem / ng, grp = rem - chunk * ng;  // (row chunk, query group), group fastest
    const int q_begin = (int)((int64_t)grp * c / ng), q_end = (int)((int64_t)(grp + 1) * c / ng);
    const int nqi = q_end - q_begin;
    const int64_t r0 = lr0 + (int64_t)chunk * MF_CH;
    const int64_t r1 = r0 + MF_CH < lr1 ? r0 + MF_CH : lr1;
    const int boff = bucket_off[l] + q_begin;
    const int nqt = (nqi + 15) >> 4;

    // ---- the item's queries → LDS: [query][stride] fp32, dims ≥ d zero ----
    const int stride = mf_stride(d);
    const int nf4 = mf_nsub(d) * 4;
    for (int t = threadIdx.x; t < nqi * nf4; t += MF_THREADS) {
        const int q = t / nf4, f = t - (t / nf4) * nf4;
        const float *src = Q + (int64_t)(bucket[boff + q] / nprobe) * d;
        mf_f32x4 v = mf_f32x4{0.f, 0.f, 0.f, 0.f};
        if (4 * f < d) v = *reinterpret_cast<const mf_f32x4 *>(src + 4 * f);
        *reinterpret_cast<mf_f32x4 *>(smem + q * stride + 4 * f) = v;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t tp0 = tpass_off[l] + (int64_t)chunk * (MF_CH / MF_PASS);
#define MF_ARGS d, codes_t, tp0, xn, r0, r1, nqi, smem, stride, qn, qb, bucket, boff, nprobe, slot_off, chunk, k, sub, smem, \
                qbound, part_d, part_i
#define MF_QN(QTV)                                                                                          \
    float qn[QTV][4];                                                                                       \
    unsigned qb[QTV][4];                                                                                    \
    _Pragma("unroll") for (int qt = 0; qt < QTV; ++qt) _Pragma("unroll") for (int v = 0; v < 4; ++v) {      \
        const int q = qt * 16 + 4 * g + v;                                                                  \
        const int qi = q < nqi ? bucket[boff + q] / nprobe : 0;                                             \
        qn[qt][v] = (!IP && q < nqi) ? qnorm[qi] : 0.f;                                                     \
        qb[qt][v] = q < nqi ? __atomic_load_n(qbound + qi, __ATOMIC_RELAXED) : 0xffffffffu;                 \
    }
    if (nqt <= 1) {
        MF_QN(1)
        mf_item<1, IP>(MF_ARGS);
    } else if (nqt == 2) {
        MF_QN(2)
        mf_item<2, IP>(MF_ARGS);
    } else {
        MF_QN(3)
        mf_item<3, IP>(MF_ARGS);
    }
#undef MF_QN
#undef MF_ARGS
}

// Tiled copy of the list-contiguous row-major codes: one block per 32-row pass (list found by binary
// search over the pass offsets); element (pass, step s, tile r, lane (g, m), e) = row 32·p + 16r + m
// of the list, dim 16s + 4g + e, zero past the list's end and past d.
__global__ void __launch_bounds__(256)
ivf_tile_codes(const float *__restrict__ codes, const int64_t *__restrict__ list_off, const int *__restrict__ list_len,
               const int64_t *__restrict__ tpass_off, int nlist, int d, int nsub, float *__restrict__ dst,
               const int64_t *__restrict__ pass_ids) {
    const int64_t pass = pass_ids ? pass_ids[blockIdx.x] : (int64_t)blockIdx.x;
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tpass_off[mid] <= pass) lo = mid; else hi = mid - 1;
    }
    const int64_t len = list_len[lo];
    const int64_t prow = (pass - tpass_off[lo]) * MF_PASS;
    const int nf4 = nsub * MF_RT * 64;
    for (int t = threadIdx.x; t < nf4; t += 256) {
        const int s = t / (MF_RT * 64), rem = t - s * (MF_RT * 64);
        const int r = rem >> 6, lane = rem & 63, g = lane >> 4, m = lane & 15;
        const int64_t row = prow + 16 * r + m;
        const int dim = 16 * s + 4 * g;
        mf_f32x4 v = mf_f32x4{0.f, 0.f, 0.f, 0.f};
        if (row < len && dim < d) v = *reinterpret_cast<const mf_f32x4 *>(codes + (list_off[lo] + row) * (int64_t)d + dim);
        *reinterpret_cast<mf_f32x4 *>(dst + (pass * nf4 + t) * 4) = v;
    }
}

int64_t ivf_mfma_pass_floats(int d) { return (int64_t)mf_nsub(d) * MF_RT * 256; }

void launch_ivf_tile_codes(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                           int nlist, int64_t total_pass, int d, float *dst, hipStream_t st, const int64_t *pass_ids) {
    if (total_pass <= 0) return;
    HIPANN_REQUIRE(d % 4 == 0 && (uintptr_t)codes % 16 == 0, "tiled codes need d % 4 == 0 and 16-B aligned rows");
    HIPANN_REQUIRE(total_pass < (int64_t)0x7fffffff, "too many passes");
    hipLaunchKernelGGL(ivf_tile_codes, dim3((unsigned)total_pass), dim3(256), 0, st, codes, list_off, list_len,
                       tpass_off, nlist, d, mf_nsub(d), dst, pass_ids);
    HIPANN_CHECK(hipGetLastError());
}

bool ivf_mfma_supported(const float *Q, int d, const float *codes, int k) {
    return (d % 4 == 0) && ((uintptr_t)Q % 16 == 0) && ((uintptr_t)codes % 16 == 0) && k >= 1 && k <= MF_KMAX &&
           mf_group(d) >= 16;
}

int ivf_mfma_group(int d) { return mf_group(d); }

void launch_ivf_scan_mfma(const float *Q, const float *qn, int d, int metric, const float *codes_t,
                          const int64_t *tpass_off, const float *xn,
                          const int64_t *list_off, const int *list_len, const int *cnt, const int *bucket_off,
                          const int *item_off, const int *bucket, const int *slot_off, int nlist, int nprobe, int k,
                          int64_t max_items, unsigned *qbound, float *pd, int *pi, hipStream_t st, int sub) {
    if (max_items <= 0) return;
    HIPANN_REQUIRE(max_items < (int64_t)0x7fffffff, "too many IVF work items");
    HIPANN_REQUIRE(ivf_mfma_supported(Q, d, codes_t, k), "MFMA IVF scan needs d % 4 == 0, 16-B aligned data, k <= 16");
    HIPANN_REQUIRE(metric == kIP || (qn && xn), "decomposed L2 scan needs query and row norms");
    const int group = mf_group(d);
    const size_t merge = (size_t)(MF_WAVES / 2) * MF_QTMAX * 4 * 64 * sizeof(float2);  // end-of-item scratch
    const size_t smem = std::max((size_t)group * mf_stride(d) * 4, merge);
    dim3 grid((unsigned)max_items), block(MF_THREADS);
#define MF_LAUNCH_ARGS Q, qn, d, codes_t, tpass_off, xn, list_off, list_len, cnt, bucket_off, item_off, bucket, slot_off, nlist, nprobe, group, k, \
                       sub, qbound, pd, pi
    if (metric == kIP) hipLaunchKernelGGL((ivf_scan_mfma<true>), grid, block, smem, st, MF_LAUNCH_ARGS);
    else hipLaunchKernelGGL((ivf_scan_mfma<false>), grid, block, smem, st, MF_LAUNCH_ARGS);
#undef MF_LAUNCH_ARGS
    HIPANN_CHECK(hipGetLastError());
}


// ================================================================================================
// Split-bf16 variant (forms kFormSplit3 / kFormSplit2): the same item / pass / ring / selection
// structure, but q·x runs on v_mfma_f32_16x16x32_bf16 (16× the fp32 matrix rate) over an NP-term
// bf16 split of both operands, x = x₁ + x₂ (+ x₃), each term the round-to-nearest bf16 of what the
// previous ones leave (exact fp32 subtractions):
//   NP = 3: products x₁y₁ + x₁y₂ + x₂y₁ + x₁y₃ + x₃y₁ + x₂y₂ (every term ≥ 2⁻²⁴ relative), the
//           dropped ones ≤ 2⁻²⁶ relative — fp32-level products, fp32 accumulation;
//   NP = 2: x₁y₁ + x₁y₂ + x₂y₁, ≈ 2⁻¹⁶ relative per product (bf16x3 in the usual naming).
// The item's queries are split once into LDS ([query][term][32-dim super-step][g][8 bf16]); rows are
// split in registers as they arrive, once per item for all of its queries.  k-slot order inside a
// super-step follows the tiled codes: lane (g, m) holds dims 32S + 4g + j and 32S + 16 + 4g + j
// (j < 4) of row m — the same order is used for the query terms, so any permutation of dims is
// harmless (q·x does not depend on it).
typedef __bf16 mb_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 mb_bf16x2 __attribute__((ext_vector_type(2)));
typedef float mb_f32x2 __attribute__((ext_vector_type(2)));
constexpr int MB_PS = MF_P / 2;  // super-steps (two 16-dim steps) in flight per wave

__device__ __forceinline__ unsigned mb_pack(float a, float b) {
    const mb_bf16x2 v = __builtin_convertvector((mb_f32x2){a, b}, mb_bf16x2);
    return __builtin_bit_cast(unsigned, v);
}
// bf16 pair → the two fp32 values (low half first)
__device__ __forceinline__ float mb_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float mb_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

template <int NP>
struct MbTerms {
    uint4 t[NP];  // term j: 8 bf16 (k-slot order), two per dword
};
// Split 8 fp32 (k-slot order: a = slots 0-3, b = slots 4-7) into NP bf16 terms.
template <int NP>
__device__ __forceinline__ MbTerms<NP> mb_split(const mf_f32x4 &a, const mf_f32x4 &b) {
    MbTerms<NP> o;
    // pairs as packed fp32 (v_pk_add_f32 does both subtractions of a pair)
    mb_f32x2 x[4] = {{a[0], a[1]}, {a[2], a[3]}, {b[0], b[1]}, {b[2], b[3]}};
    unsigned w[NP][4];
#pragma unroll
    for (int j = 0; j < NP; ++j)
#pragma unroll
        for (int pr = 0; pr < 4; ++pr) {
            const unsigned pk = mb_pack(x[pr][0], x[pr][1]);
            w[j][pr] = pk;
            if (j + 1 < NP) x[pr] -= (mb_f32x2){mb_lo(pk), mb_hi(pk)};
        }
#pragma unroll
    for (int j = 0; j < NP; ++j) o.t[j] = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
    return o;
}
__host__ __device__ inline int mb_nsuper(int d) { return mf_nsub(d) / 2; }  // mf_nsub is a multiple of 6
// LDS dwords per query for one of NH dim phases: NP terms × super-steps/NH × 4 groups × 4 dwords, + 8
// (≡ 8 mod 64)
__host__ __device__ inline int mb_stride(int d, int np, int nh) { return np * (mb_nsuper(d) / nh) * 16 + 8; }
inline int mb_group_nh(int d, int np, int nh) {
    const int g = (int)(MF_LDS_MAX / ((size_t)mb_stride(d, np, nh) * 4)) / 16 * 16;
    return g < 16 * MF_QTMAX ? g : 16 * MF_QTMAX;
}
// Dim phases: the whole split query image in LDS when 48 queries fit (NH = 1), else the image of one
// half of the dims at a time (NH = 2: 3 terms × 768 dims × 48 queries = 221 KiB > 160 KiB of LDS),
// swapped between the halves of every 32-row pass (needs MB_PS | super-steps per half).
// Measured at 10M × 768 (nprobe 32 of 1024, 3 terms): NH = 2 with 48-query items 7.19 ms against NH = 1
// with 32-query items 6.28 ms — the per-pass image swaps (block barriers, L2 → LDS refills) cost more
// than the second group's row re-reads, so NH = 2 is opt-in (HIPANN_IVF_PHASES=2, tuning only).
inline int mb_phases(int d, int np) {
    static const int want = [] { const char *e = std::getenv("HIPANN_IVF_PHASES"); return e ? std::atoi(e) : 1; }();
    if (want < 2 || mb_group_nh(d, np, 1) >= 16 * MF_QTMAX) return 1;
    return mb_nsuper(d) % (2 * MB_PS) == 0 ? 2 : 1;
}
inline int mb_group(int d, int np) { return mb_group_nh(d, np, mb_phases(d, np)); }

__device__ __forceinline__ mf_f32x4 mb_mfma(const uint4 &a, const uint4 &b, const mf_f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(mb_bf16x8, a), __builtin_bit_cast(mb_bf16x8, b),
                                                   c, 0, 0, 0);
}

// Copy the item's queries' split terms for dim phase h (super-steps [h·nsup/NH, (h+1)·nsup/NH)) from the
// batch's split image qsplit [query][term][super-step][g][4 dwords] into LDS [query][term][S][g][4].
template <int NP, int NH>
__device__ __forceinline__ void mb_fill(unsigned *qs, const uint4 *__restrict__ qsplit, int nsup, int stride, int h,
                                        int nqi, const int *__restrict__ bucket, int boff, int nprobe) {
    const int nsh = nsup / NH;
    const int per_q = NP * nsh * 4;
    for (int t = threadIdx.x; t < nqi * per_q; t += MF_THREADS) {
        const int q = t / per_q, rr = t - q * per_q;
        const int j = rr / (nsh * 4), r2 = rr - j * (nsh * 4);
        const int Sl = r2 >> 2, gg = r2 & 3;
        const int gq = bucket[boff + q] / nprobe;
        const uint4 v = qsplit[(((int64_t)gq * NP + j) * nsup + h * nsh + Sl) * 4 + gg];
        *reinterpret_cast<uint4 *>(qs + q * stride + ((j * nsh + Sl) * 4 + gg) * 4) = v;
    }
}

template <int QT, bool IP, int NP, int NH>
__device__ __forceinline__ void mb_item(int d, const float *__restrict__ codes_t, int64_t tp0,
                                        const float *__restrict__ xn, int64_t r0, int64_t r1, int nqi,
                                        unsigned *__restrict__ qs, int stride, const uint4 *__restrict__ qsplit,
                                        const float (&qn)[QT][4],
                                        const unsigned (&qb)[QT][4], const int *__restrict__ bucket, int boff,
                                        int nprobe, const int *__restrict__ slot_off, int chunk, int k, int sub, float *smem,
                                        unsigned *__restrict__ qbound, float *__restrict__ part_d,
                                        int *__restrict__ part_i) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = lane & 15, g = lane >> 4;
    const int nsub = mf_nsub(d);
    const int nsup = nsub / 2;
    const int nsh = nsup / NH;  // super-steps per dim phase
    const int npass_all = (int)ceil_div(r1 - r0, MF_PASS);
    const int npass = npass_all > wave ? (npass_all - wave + MF_WAVES - 1) / MF_WAVES : 0;
    // with NH > 1 every wave walks the same number of pass slots (the image swaps are block-wide)
    const int nslots = NH > 1 ? (int)ceil_div(npass_all, MF_WAVES) : npass;

    bool qv[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) qv[qt][v] = qt * 16 + 4 * g + v < nqi;
    uint64_t lst[QT][4], thr[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint64_t b = ((uint64_t)qb[qt][v] << 32) | MF_PAD_ID;
            lst[qt][v] = m < k ? b : MF_EMPTY;
            thr[qt][v] = b;
        }

    auto row_of = [&](int i, int r) -> int64_t {
        const int64_t row = r0 + (int64_t)(wave + MF_WAVES * i) * MF_PASS + 16 * r + m;
        return row < r1 ? row : r1 - 1;
    };
    const int ilast = npass > 0 ? npass - 1 : 0;
    const float *rp;
    int ld_i = 0, ld_s = 0;  // stream position (16-dim steps), wave-uniform
    auto set_pass = [&](int i) { rp = codes_t + ((tp0 + wave + MF_WAVES * i) * nsub) * (MF_RT * 256) + 4 * lane; };
    auto next_load = [&](mf_f32x4 (&dst)[MF_RT]) {
        const int s = ld_i <= ilast ? ld_s : nsub - 1;
#pragma unroll
        for (int r = 0; r < MF_RT; ++r)
            dst[r] = *reinterpret_cast<const mf_f32x4 *>(rp + (int64_t)s * (MF_RT * 256) + r * 256);
        if (++ld_s == nsub) {
            ld_s = 0;
            ++ld_i;
            set_pass(ld_i <= ilast ? ld_i : ilast);
        }
    };

    mf_f32x4 ring[MB_PS][2][MF_RT];  // [super-step slot][half][row tile]
    float xnr[MF_RT] = {0.f, 0.f};
    if (npass > 0) {
        set_pass(0);
#pragma unroll
        for (int p = 0; p < MB_PS; ++p) {
            next_load(ring[p][0]);
            next_load(ring[p][1]);
        }
        if (!IP) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr[r] = xn[row_of(0, r)];
        }
    }
    const unsigned *qrow[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) qrow[qt] = qs + (qt * 16 + m) * stride + 4 * g;

    mf_f32x4 acc[QT][MF_RT];
    for (int i = 0; i < nslots; ++i) {
        const bool has = i < npass;  // wave-uniform; false only in the last slot of a ragged item
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) acc[qt][r] = mf_f32x4{0.f, 0.f, 0.f, 0.f};
        float xnr_next[MF_RT] = {0.f, 0.f};
        if (!IP && has) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr_next[r] = xn[row_of(i + 1 <= ilast ? i + 1 : ilast, r)];
        }
        for (int h = 0; h < NH; ++h) {
        if (NH > 1) {
            __syncthreads();  // every wave is done with the previous phase's image
            mb_fill<NP, NH>(qs, qsplit, nsup, stride, h, nqi, bucket, boff, nprobe);
            __syncthreads();
        }
        if (has)
        for (int S0 = 0; S0 < nsh; S0 += MB_PS) {
#pragma unroll
            for (int p = 0; p < MB_PS; ++p) {
                const int S = S0 + p;
                uint4 qa[QT][NP];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int j = 0; j < NP; ++j)
                        qa[qt][j] = *reinterpret_cast<const uint4 *>(qrow[qt] + (j * nsh + S) * 16);
                MbTerms<NP> xb[MF_RT];
#pragma unroll
                for (int r = 0; r < MF_RT; ++r) xb[r] = mb_split<NP>(ring[p][0][r], ring[p][1][r]);
                next_load(ring[p][0]);
                next_load(ring[p][1]);
                // products, small terms first per accumulator chain position (independent chains
                // interleave: consecutive MFMAs hit different accumulators)
#pragma unroll
                for (int t = 0; t < (NP == 3 ? 6 : 3); ++t) {
                    const int ja = NP == 3 ? (t == 0 ? 1 : t == 1 ? 0 : t == 2 ? 2 : t == 3 ? 0 : t == 4 ? 1 : 0)
                                           : (t == 0 ? 1 : t == 1 ? 0 : 0);
                    const int jb = NP == 3 ? (t == 0 ? 1 : t == 1 ? 2 : t == 2 ? 0 : t == 3 ? 1 : t == 4 ? 0 : 0)
                                           : (t == 0 ? 0 : t == 1 ? 1 : 0);
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int r = 0; r < MF_RT; ++r) acc[qt][r] = mb_mfma(qa[qt][ja], xb[r].t[jb], acc[qt][r]);
                }
            }
        }
        }  // dim phases
        if (!has) continue;
        const int64_t prow0 = r0 + (int64_t)(wave + MF_WAVES * i) * MF_PASS;
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) {
            const int64_t row = prow0 + 16 * r + m;
            const bool rok = row < r1;
            const unsigned rid = rok ? (unsigned)row : MF_PAD_ID;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    float key;
                    if (IP) {
                        key = -acc[qt][r][v];
                    } else {
                        key = fmaf(-2.f, acc[qt][r][v], qn[qt][v] + xnr[r]);
                        key = key < 0.f ? 0.f : key;
                    }
                    const bool ok = rok && qv[qt][v];
                    uint64_t cp = ok ? (((uint64_t)mf_sortable(key) << 32) | rid) : MF_EMPTY;
                    if (__ballot(cp < thr[qt][v])) {
                        row_sort16(cp, m);
                        row_merge16(lst[qt][v], cp, m);
                        thr[qt][v] = row_kth(lst[qt][v], k - 1, g);
                    }
                }
        }
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) xnr[r] = xnr_next[r];
    }

    mf_finish_item<QT>(lst, smem, nqi, bucket, boff, nprobe, slot_off, chunk, k, sub, qbound, part_d, part_i);
}

template <bool IP, int NP, int NH>
__global__ void __launch_bounds__(MF_THREADS, MF_WAVES / 4)
ivf_scan_mfma_bf(const uint4 *__restrict__ qsplit, const float *__restrict__ qnorm, int d, const float *__restrict__ codes_t,
                 const int64_t *__restrict__ tpass_off, const float *__restrict__ xn,
                 const int64_t *__restrict__ list_off, const int *__restrict__ list_len, const int *__restrict__ cnt, const int *__restrict__ bucket_off,
                 const int *__restrict__ item_off, const int *__restrict__ bucket, const int *__restrict__ slot_off,
                 int nlist, int nprobe, int group, int k, int sub, unsigned *__restrict__ qbound, float *__restrict__ part_d,
                 int *__restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int total = item_off[nlist];
    if ((int)blockIdx.x >= total) return;
    const int item = xcd_remap((int)blockIdx.x, total);
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int64_t lr0 = list_off[l], lr1 = lr0 + list_len[l];
    const int c = cnt[l];
    const int ng = (c + group - 1) / group;
    const int rem = item - item_off[l];
    const int chunk = rem / ng, grp = rem - chunk * ng;
    const int q_begin = (int)((int64_t)grp * c / ng), q_end = (int)((int64_t)(grp + 1) * c / ng);
    const int nqi = q_end - q_begin;
    const int64_t r0 = lr0 + (int64_t)chunk * MF_CH;
    const int64_t r1 = r0 + MF_CH < lr1 ? r0 + MF_CH : lr1;
    const int boff = bucket_off[l] + q_begin;
    const int nqt = (nqi + 15) >> 4;

    // ---- the item's queries' split terms → LDS [query][term][S][g][8 bf16] (all dims, or per phase) ----
    unsigned *qs = reinterpret_cast<unsigned *>(smem);
    const int stride = mb_stride(d, NP, NH);
    if (NH == 1) mb_fill<NP, 1>(qs, qsplit, mb_nsuper(d), stride, 0, nqi, bucket, boff, nprobe);
    __syncthreads();

    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int64_t tp0 = tpass_off[l] + (int64_t)chunk * (MF_CH / MF_PASS);
#define MB_ARGS d, codes_t, tp0, xn, r0, r1, nqi, qs, stride, qsplit, qn, qb, bucket, boff, nprobe, slot_off, chunk, k, sub, smem, \
                qbound, part_d, part_i
#define MB_QN(QTV)                                                                                          \
    float qn[QTV][4];                                                                                       \
    unsigned qb[QTV][4];                                                                                    \
    _Pragma("unroll") for (int qt = 0; qt < QTV; ++qt) _Pragma("unroll") for (int v = 0; v < 4; ++v) {      \
        const int q = qt * 16 + 4 * g + v;                                                                  \
        const int qi = q < nqi ? bucket[boff + q] / nprobe : 0;                                             \
        qn[qt][v] = (!IP && q < nqi) ? qnorm[qi] : 0.f;                                                     \
        qb[qt][v] = q < nqi ? __atomic_load_n(qbound + qi, __ATOMIC_RELAXED) : 0xffffffffu;                 \
    }
    if (nqt <= 1) {
        MB_QN(1)
        mb_item<1, IP, NP, NH>(MB_ARGS);
    } else if (nqt == 2) {
        MB_QN(2)
        mb_item<2, IP, NP, NH>(MB_ARGS);
    } else {
        MB_QN(3)
        mb_item<3, IP, NP, NH>(MB_ARGS);
    }
#undef MB_QN
#undef MB_ARGS
}

// The batch's queries split once into NP bf16 terms: qsplit [query][term][super-step][g][8 bf16], k-slot
// order of the tiled codes (dims 32S + 4g + j and 32S + 16 + 4g + j, j < 4; zero past d).
template <int NP>
__global__ void __launch_bounds__(256) ivf_split_queries(const float *__restrict__ Q, int64_t nq, int d, int nsup,
                                                         uint4 *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nq * nsup * 4) return;
    const int64_t q = t / (nsup * 4);
    const int rr = (int)(t - q * (nsup * 4));
    const int S = rr >> 2, gg = rr & 3;
    const float *src = Q + q * d;
    const int d0 = 32 * S + 4 * gg, d1 = d0 + 16;
    mf_f32x4 a = mf_f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
    if (d0 < d) a = *reinterpret_cast<const mf_f32x4 *>(src + d0);
    if (d1 < d) b = *reinterpret_cast<const mf_f32x4 *>(src + d1);
    const MbTerms<NP> sp = mb_split<NP>(a, b);
#pragma unroll
    for (int j = 0; j < NP; ++j) out[((q * NP + j) * nsup + S) * 4 + gg] = sp.t[j];
}

int ivf_mfma_bf_group(int d, int np) { return mb_group(d, np); }

int64_t ivf_mfma_bf_qsplit_bytes(int64_t nq, int d, int np) { return nq * np * mb_nsuper(d) * 64; }

bool ivf_mfma_bf_supported(const float *Q, int d, const float *codes, int k, int np) {
    return ivf_mfma_supported(Q, d, codes, k) && mb_group(d, np) >= 16;
}

void launch_ivf_scan_mfma_bf(int np, const float *Q, int64_t nq, void *qsplit, const float *qn, int d, int metric,
                             const float *codes_t, const int64_t *tpass_off, const float *xn, const int64_t *list_off,
                             const int *list_len, const int *cnt, const int *bucket_off, const int *item_off, const int *bucket,
                             const int *slot_off, int nlist, int nprobe, int k, int64_t max_items, unsigned *qbound,
                             float *pd, int *pi, hipStream_t st, int sub) {
    if (max_items <= 0 || nq <= 0) return;
    HIPANN_REQUIRE(np == 2 || np == 3, "split-bf16 scan: 2 or 3 terms");
    HIPANN_REQUIRE(max_items < (int64_t)0x7fffffff, "too many IVF work items");
    HIPANN_REQUIRE(qsplit, "split-bf16 scan: no query image buffer");
    HIPANN_REQUIRE(ivf_mfma_bf_supported(Q, d, codes_t, k, np), "split-bf16 IVF scan needs d % 4 == 0, 16-B aligned data, k <= 16");
    HIPANN_REQUIRE(metric == kIP || (qn && xn), "decomposed L2 scan needs query and row norms");
    const int nsup = mb_nsuper(d);
    const int64_t nthr = nq * nsup * 4;
    uint4 *qs = static_cast<uint4 *>(qsplit);
    if (np == 3) hipLaunchKernelGGL(ivf_split_queries<3>, dim3((unsigned)ceil_div(nthr, 256)), dim3(256), 0, st, Q, nq, d, nsup, qs);
    else hipLaunchKernelGGL(ivf_split_queries<2>, dim3((unsigned)ceil_div(nthr, 256)), dim3(256), 0, st, Q, nq, d, nsup, qs);
    const int nh = mb_phases(d, np);
    const int group = mb_group(d, np);
    const size_t merge = (size_t)(MF_WAVES / 2) * MF_QTMAX * 4 * 64 * sizeof(float2);
    const size_t smem = std::max((size_t)group * mb_stride(d, np, nh) * 4, merge);
    dim3 grid((unsigned)max_items), block(MF_THREADS);
#define MB_LAUNCH_ARGS qs, qn, d, codes_t, tpass_off, xn, list_off, list_len, cnt, bucket_off, item_off, bucket, slot_off, nlist, nprobe, \
                       group, k, sub, qbound, pd, pi
#define MB_LAUNCH(NP_, NH_)                                                                                         \
    do {                                                                                                            \
        if (metric == kIP) hipLaunchKernelGGL((ivf_scan_mfma_bf<true, NP_, NH_>), grid, block, smem, st, MB_LAUNCH_ARGS); \
        else hipLaunchKernelGGL((ivf_scan_mfma_bf<false, NP_, NH_>), grid, block, smem, st, MB_LAUNCH_ARGS);       \
    } while (0)
    if (np == 3) {
        if (nh == 2) MB_LAUNCH(3, 2); else MB_LAUNCH(3, 1);
    } else {
        if (nh == 2) MB_LAUNCH(2, 2); else MB_LAUNCH(2, 1);
    }
#undef MB_LAUNCH
#undef MB_LAUNCH_ARGS
    HIPANN_CHECK(hipGetLastError());
}


// ================================================================================================
// fp16-image variant (form kFormHalfExact): the list scan reads HALF the bytes of the fp32 forms.
// The rows are stored once as a tiled fp16 image of x·s (s = 2^(14 − e), max|x| = f·2^e, f ∈ [½, 1):
// every scaled element ≤ 2^14, far inside fp16's range), round to nearest even, subnormal results
// flushed to zero; each query is scaled the same way (t = 2^(14 − e_q)) and split into two fp16 terms
// q·t = h + l (+ ≤ 2⁻²² relative), so q·x ≈ (h + l)·x̂ / (t·s) on v_mfma_f32_16x16x32_f16 (fp16 × fp16
// products are exact in fp32, fp32 accumulation) — or, in the one-term items that are the default since r06
// (mh_wide_mode), h·x̂ / (t·s) with the query's own one-term residual ‖q − h/t‖ in the bound.  The other error is
// the rows' own fp16 rounding, |q·(x − x̂/s)| ≤ ‖q‖·‖x − x̂/s‖, and the scan is a FILTER: it keeps the 16 best per
// (query, list, chunk) like form 5, ivf_rerank_topk recomputes them in FAISS's direct fp32 form and
// proves with the measured residuals (largest row residual, this query's split residual) that no
// pruned row reaches the top-k; failing queries re-run on the device in the direct form.
// Image layout (per list, 32-row passes as codes_t): [pass][32-dim super-step S][row tile r][lane (g, m)]
// [8 halves] = row 16r + m, dims 32S + 4g + j and 32S + 16 + 4g + j (j < 4) — the k-slot order of the
// split-bf16 variant, so a wave load is 1 KiB contiguous and a pass of d = 768 is 48 KiB.
typedef _Float16 mh_f16x8 __attribute__((ext_vector_type(8)));
#ifndef HIPANN_MH_P
#define HIPANN_MH_P 6
#endif
#ifndef HIPANN_MH_FOLLOW
// 1 (tuning builds, with HIPANN_IVF_FOLLOW=1): items start at the round another query group of their chunk last
// published.  Measured and left out: same box, alternating (tools/gpu_r06_follow.sh, profiles/r06/
// ivf_follow_ab_r06.txt) the SURVEY mixture's scan 5.14 / 5.25 ms against 5.23 / 5.24 (runtime off) and 5.18 / 5.20
// (compiled out) — within the noise; the rotation's scalar registers spill to VGPR lanes for nothing
#define HIPANN_MH_FOLLOW 0
#endif
#ifndef HIPANN_MH_EARLY
#define HIPANN_MH_EARLY 1  // issue the item's first row loads before waiting for its query fill (0: fill, barrier, loads)
#endif
#ifndef HIPANN_MH_NT
#define HIPANN_MH_NT 1  // non-temporal row loads (the image is read once per batch): 2.67 -> 2.59 ms at 10M x 768
#endif
constexpr int MH_P = HIPANN_MH_P;  // super-steps in flight per wave: 6 × 2 row tiles × 16 B = 192 B per lane
__host__ __device__ inline int mh_nsup(int d) { return (int)ceil_div(ceil_div(d, 32), MH_P) * MH_P; }
// LDS dwords per query: NT terms × super-steps × 4 groups × 4 dwords, + 8 (≡ 8 mod 64: conflict-free)
__host__ __device__ inline int mh_stride(int d, int nt = 2) { return nt * mh_nsup(d) * 16 + 8; }
inline int mh_group(int d) {
    const int g = (int)(MF_LDS_MAX / ((size_t)mh_stride(d) * 4)) / 16 * 16;
    return g < 16 * MF_QTMAX ? g : 16 * MF_QTMAX;
}
// Wide items (lists probed by more queries than one two-term group holds): the queries' high fp16 term only, so
// twice the queries fit the LDS (96 at d = 768) and the list's rows are streamed half as often; MFMAs per row and
// query halve too.  The price is the query's own split residual: ‖q − h/t‖ (≈ 2⁻¹² relative) instead of
// ‖q − (h + l)/t‖ (≈ 2⁻²³), which the scan hands to the rerank's bound for every query of a wide item.
// On SURVEY §8(d)'s mixture (σ 0.8, nprobe 16) popular lists are probed by up to ~400 queries: 9 two-term
// groups re-read each 2048-row chunk, 36 % of it from L2 (profiles/r06/mixture_scan_pmc_r06.txt).
constexpr int MH_QTW = 6;  // query tiles of a wide item
inline int mh_group_wide(int d) {  // the image + (‖q‖², 1/(t·s)) per query
    const int g = (int)(MF_LDS_MAX / ((size_t)mh_stride(d, 1) * 4 + 8)) / 16 * 16;
    return g < 16 * MH_QTW ? g : 16 * MH_QTW;
}
// HIPANN_IVF_WIDE: 2 (default) every item one-term (narrow size 0: groups of up to 96 queries); 1 (A/B) two-term items
// for lists probed by ≤ 48 queries, one-term above; 0 (A/B) every item two-term.  Same box, alternating
// (tools/gpu_r06_wide.sh MODES="1 2"): the headline 382.2K / 382.0K → 395.9K / 395.9K QPS (scan 2.553 → 2.491 ms: half
// the MFMAs and LDS reads per row and query), the mixture unchanged, 0 flagged queries in both
inline int mh_wide_mode() {
    static const int mode = [] { const char *e = std::getenv("HIPANN_IVF_WIDE"); return e ? std::atoi(e) : 2; }();
    return mode;
}
// GEMM items (lists probed by more queries than a wide item holds): up to MG_Q queries, database rows and queries both
// staged through LDS by LDS-DMA (mg_item below).  HIPANN_IVF_GEMM=1 (A/B) enables them; off by default: measured
// slower, same box, alternating (tools/gpu_r06_gemm.sh, profiles/r06/ivf_gemm_items_ab_r06.txt) — the SURVEY mixture's
// scan 5.17 → 8.32 ms at nprobe 16, intrinsic dimension 32 at nprobe 128 185K → 112K QPS.  The item streams its rows
// with too little in flight: vector-memory loads retire in issue order, so the rows (HBM) and the query slices (L2)
// share one lead, and four 24 KiB stages keep only 24 KiB of rows in flight per CU against the wide items' 96 KiB.
constexpr int MG_Q = 256;
inline bool mg_enabled() {
    static const bool on = [] { const char *e = std::getenv("HIPANN_IVF_GEMM"); return e && std::atoi(e); }();
    return on;
}
// the packed group of the plan and the scan (narrow | wide << 8 | GEMM << 16: ivf_ngroups, common.hpp)
inline int mh_group_packed(int d) {
    const int g = mh_group(d), w = mh_group_wide(d);
    if (!mh_wide_mode() || w <= g || g < 16) return g;
    const int gm = mg_enabled() && w >= 16 ? MG_Q << 16 : 0;
    return (mh_wide_mode() == 2 ? 0 : g) | (w << 8) | gm;
}

// fp32 → fp16 round to nearest even; subnormal results flushed to zero (the MFMA sees only normal
// values or zero whatever its denormal mode, and the residuals are measured against exactly this)
__device__ __forceinline__ unsigned short mh_half_bits(float v) {
    const _Float16 h = (_Float16)v;
    return __builtin_fabsf((float)h) < 0x1p-14f ? (unsigned short)0 : __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float mh_val(unsigned short b) { return (float)__builtin_bit_cast(_Float16, b); }
__device__ __forceinline__ unsigned mh_pack(float a, float b) {
    return (unsigned)mh_half_bits(a) | ((unsigned)mh_half_bits(b) << 16);
}

__device__ __forceinline__ mf_f32x4 mh_mfma(const uint4 &a, const uint4 &b, const mf_f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(mh_f16x8, a), __builtin_bit_cast(mh_f16x8, b), c,
                                                  0, 0, 0);
}

// ---- int8 image (form kFormI8Exact) -------------------------------------------------------------------------
// The lists as a tiled int8 image with one scale per row (s = max|x| / 127, x̂ = clamp(rint(x / s), ±127): the Flat
// form 5's quantizer, i8_quant) — a quarter of the fp32 rows' bytes, half the fp16 image's — scanned on
// v_mfma_i32_16x16x64_i8 (exact int32 sums) against int8 queries (their own scale); key = ‖q‖² + ‖x‖² − 2·s_q·s_x·sum.
// Same geometry as the fp16 image with 64-dim super-steps: [pass][S][row tile r][lane (g, m)][16 B] = row 16r + m,
// dims 64S + 16g .. +15 (the queries' units use the same lane order, so the MFMA pairs equal k-slots whatever its
// internal k mapping).  The filter is coarser (≈ 2⁻⁸ relative): the scan always keeps per-wave sub-lists and the
// rerank takes 64 candidates, certified with the int8 residuals (max row ‖x − s·x̂‖, the query's own).
typedef int mf_i32x4 __attribute__((ext_vector_type(4)));
__host__ __device__ inline int mi_nsup(int d) { return (int)ceil_div(ceil_div(d, 64), MH_P) * MH_P; }
__device__ __forceinline__ int mi_quant(float x, float s) {
    return s > 0.f ? (int)fminf(fmaxf(rintf(x / s), -127.f), 127.f) : 0;
}
__device__ __forceinline__ uint4 mi_units(const float *x, int dim0, int d, float s) {  // 16 dims → 16 int8
    unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int v = dim0 + i < d ? mi_quant(x[dim0 + i], s) : 0;
        w[i >> 2] |= ((unsigned)v & 0xffu) << (8 * (i & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}
// max|x| / 127 of a row (0 for a zero or non-finite row: its units are 0 and its residual +inf, see mi_resid)
__device__ __forceinline__ float mi_row_scale(const float *x, int d, int lane) {
    float mx = 0.f;
    for (int e = lane; e < d; e += 64) mx = fmaxf(mx, fabsf(x[e]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    return mx > 0.f && mx < 3.0e38f ? mx / 127.f : (mx == 0.f ? 0.f : -1.f);
}

// one block per 32-row pass (list by binary search over the pass offsets, as ivf_tile_half): the rows' scales (into
// xs8 at their CSR rows) and the pass's units; rows past the list's live length: zero units, scale 0
__global__ void __launch_bounds__(256)
ivf_tile_i8(const float *__restrict__ codes, const int64_t *__restrict__ list_off, const int *__restrict__ list_len,
            const int64_t *__restrict__ tpass_off, int nlist, int d, int nsup, uint4 *__restrict__ dst,
            float *__restrict__ xs8, const int64_t *__restrict__ pass_ids) {
    const int64_t pass = pass_ids ? pass_ids[blockIdx.x] : (int64_t)blockIdx.x;
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tpass_off[mid] <= pass) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int64_t r0 = list_off[l] + (pass - tpass_off[l]) * 32, rend = list_off[l] + list_len[l];
    __shared__ float sc[32];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int rr = wave; rr < 32; rr += 4) {
        const int64_t row = r0 + rr;
        float s = 0.f;
        if (row < rend) {
            s = mi_row_scale(codes + row * (int64_t)d, d, lane);
            if (s < 0.f) s = 0.f;  // non-finite row: zero units (its residual is +inf: the rerank re-runs every query)
        }
        if (lane == 0) {
            sc[rr] = s;
            if (row < list_off[l + 1]) xs8[row] = s;
        }
    }
    __syncthreads();
    for (int u = threadIdx.x; u < nsup * MF_RT * 64; u += 256) {
        const int S = u / (MF_RT * 64), rem = u - S * (MF_RT * 64), r = rem >> 6, ln = rem & 63;
        const int rr = 16 * r + (ln & 15), g = ln >> 4;
        const int64_t row = r0 + rr;
        dst[(pass * nsup + S) * (MF_RT * 64) + rem] =
            row < rend ? mi_units(codes + row * (int64_t)d, 64 * S + 16 * g, d, sc[rr]) : make_uint4(0u, 0u, 0u, 0u);
    }
}

// max over rows of ‖x − s·x̂‖² (one wave per row; +inf for a non-finite row) as float bits
__global__ void __launch_bounds__(256) ivf_i8_residual(const float *__restrict__ codes, int64_t n, int d,
                                                       unsigned *__restrict__ out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    const float *x = codes + row * (int64_t)d;
    const float s = mi_row_scale(x, d, lane);
    float r2 = 0.f;
    if (s >= 0.f) {
        for (int e = lane; e < d; e += 64) {
            const float rr = x[e] - s * (float)mi_quant(x[e], s);
            r2 = fmaf(rr, rr, r2);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r2 += __shfl_xor(r2, o);
    } else {
        r2 = __builtin_inff();
    }
    if (lane == 0) atomicMax(out, __float_as_uint(r2));
}

// The batch's int8 queries, one wave per query: scale qs8 = max|q| / 127, residual qres8 = ‖q − qs8·q̂‖ (×1.0001; +inf
// for a non-finite query: the rerank re-runs it) and the units [q][S][g] (zero past d)
__global__ void __launch_bounds__(256) ivf_split_queries_i8(const float *__restrict__ Q, int64_t nq, int d, int nsup,
                                                            uint4 *__restrict__ out, float *__restrict__ qs8,
                                                            float *__restrict__ qres8) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    const float *x = Q + q * (int64_t)d;
    float s = mi_row_scale(x, d, lane);
    const bool fin = s >= 0.f;
    if (!fin) s = 0.f;
    float r2 = 0.f;
    for (int e = lane; e < d; e += 64) {
        const float rr = x[e] - s * (float)mi_quant(x[e], s);
        r2 = fmaf(rr, rr, r2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r2 += __shfl_xor(r2, o);
    if (lane == 0) {
        qs8[q] = s;
        qres8[q] = fin ? sqrtf(r2) * 1.0001f : __builtin_inff();
    }
    for (int u = lane; u < nsup * 4; u += 64) out[q * nsup * 4 + u] = mi_units(x, 64 * (u >> 2) + 16 * (u & 3), d, s);
}

// max |x| over cnt floats as the bits of the magnitude (unsigned order = magnitude order; any NaN
// compares above +inf, so a non-finite table is detected by bits >= 0x7f800000)
__global__ void __launch_bounds__(256) ivf_max_abs(const float *__restrict__ x, int64_t cnt, unsigned *__restrict__ out) {
    unsigned m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256)
        m = max(m, __float_as_uint(x[i]) & 0x7fffffffu);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

// one block per 32-row pass (list found by binary search over the pass offsets); zero past the
// list's end and past d
__global__ void __launch_bounds__(256)
ivf_tile_half(const float *__restrict__ codes, const int64_t *__restrict__ list_off, const int *__restrict__ list_len,
              const int64_t *__restrict__ tpass_off, int nlist, int d, int nsup, float scale, uint4 *__restrict__ dst,
              const int64_t *__restrict__ pass_ids) {
    const int64_t pass = pass_ids ? pass_ids[blockIdx.x] : (int64_t)blockIdx.x;
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tpass_off[mid] <= pass) lo = mid; else hi = mid - 1;
    }
    const int64_t len = list_len[lo];
    const int64_t prow = (pass - tpass_off[lo]) * MF_PASS;
    const int nt = nsup * MF_RT * 64;
    for (int t = threadIdx.x; t < nt; t += 256) {
        const int S = t / (MF_RT * 64), rem = t - S * (MF_RT * 64);
        const int r = rem >> 6, lane = rem & 63, g = lane >> 4, m = lane & 15;
        const int64_t row = prow + 16 * r + m;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
        if (row < len) {
            const float *src = codes + (list_off[lo] + row) * (int64_t)d;
            const int d0 = 32 * S + 4 * g, d1 = d0 + 16;
            if ((d & 3) == 0 && ((uintptr_t)codes & 15) == 0) {  // whole float4s (d0, d1 are multiples of 4)
                if (d0 < d) {
                    const float4 a = *reinterpret_cast<const float4 *>(src + d0);
                    v[0] = a.x * scale; v[1] = a.y * scale; v[2] = a.z * scale; v[3] = a.w * scale;
                }
                if (d1 < d) {
                    const float4 b = *reinterpret_cast<const float4 *>(src + d1);
                    v[4] = b.x * scale; v[5] = b.y * scale; v[6] = b.z * scale; v[7] = b.w * scale;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (d0 + j < d) v[j] = src[d0 + j] * scale;
                    if (d1 + j < d) v[4 + j] = src[d1 + j] * scale;
                }
            }
        }
        dst[pass * nt + t] = make_uint4(mh_pack(v[0], v[1]), mh_pack(v[2], v[3]), mh_pack(v[4], v[5]), mh_pack(v[6], v[7]));
    }
}

// max over rows of ‖x − x̂/s‖² (one wave per row), as float bits
__global__ void __launch_bounds__(256) ivf_half_residual(const float *__restrict__ codes, int64_t n, int d, float scale,
                                                         float inv_scale, unsigned *__restrict__ out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    float s = 0.f;
    if (row < n) {
        const float *src = codes + row * (int64_t)d;
        for (int e = lane; e < d; e += 64) {
            const float x = src[e];
            const float r = x - mh_val(mh_half_bits(x * scale)) * inv_scale;  // exact (Sterbenz / flushed: r = x)
            s = fmaf(r, r, s);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0 && row < n) atomicMax(out, __float_as_uint(s));
}

// An append block (hipann_ivf_add), one wave per row j of the block: the row into its physical CSR row dst[j] (codes,
// label, and the L2 norm launch_row_norms computed over the block — the bits a rebuild computes); rows of another
// shard's lists (dst < 0) are skipped.  The same pass folds this shard's new rows into the running maxima: stat[0] =
// max ‖x‖² (float bits), stat[1] = max |x| (magnitude bits: NaN above +inf, as ivf_max_abs), stat[2] = max fp16
// residual² ‖x − x̂/s‖² at the image's scale s (hscale > 0; ivf_half_residual's summation order).  Threads below
// nlist also publish the new live lengths (read by the re-tile that follows and by the next search).
__global__ void __launch_bounds__(256)
ivf_append_rows(const float *__restrict__ rows, const float *__restrict__ norms, const int64_t *__restrict__ dst,
                const int64_t *__restrict__ ids_in, int64_t n, int d, float *__restrict__ codes,
                int64_t *__restrict__ ids, float *__restrict__ xnorm, const int *__restrict__ newlen,
                int *__restrict__ list_len, int nlist, float hscale, unsigned *__restrict__ stat) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid < nlist) list_len[gid] = newlen[gid];
    const int lane = threadIdx.x & 63;
    if (!dst) {
        // statistics only (every row of the block; nothing written but stat) — the pre-pass whose maxima come back with
        // the coarse assignment, so the append needs no host wait of its own.  A few blocks stride over the rows and
        // reduce in the block before one atomic per statistic (one atomic per row on three words serialised: 74 µs
        // for 2048 rows)
        __shared__ unsigned red[3][4];
        const float inv = hscale > 0.f ? 1.f / hscale : 0.f;
        unsigned mn = 0, ma = 0, mr = 0;
        for (int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += (int64_t)gridDim.x * 4) {
            const float *src = rows + j * (int64_t)d;
            unsigned mabs = 0;
            float res = 0.f;
            for (int e = lane; e < d; e += 64) {
                const float x = src[e];
                mabs = max(mabs, __float_as_uint(x) & 0x7fffffffu);
                if (hscale > 0.f) {
                    const float q = x - mh_val(mh_half_bits(x * hscale)) * inv;
                    res = fmaf(q, q, res);
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                mabs = max(mabs, (unsigned)__shfl_xor((int)mabs, o));
                res += __shfl_xor(res, o);
            }
            mn = max(mn, __float_as_uint(norms[j]));
            ma = max(ma, mabs);
            mr = max(mr, __float_as_uint(res));
        }
        if (lane == 0) {
            red[0][threadIdx.x >> 6] = mn;
            red[1][threadIdx.x >> 6] = ma;
            red[2][threadIdx.x >> 6] = mr;
        }
        __syncthreads();
        if (threadIdx.x < 3 && stat) {
            const unsigned v = max(max(red[threadIdx.x][0], red[threadIdx.x][1]), max(red[threadIdx.x][2], red[threadIdx.x][3]));
            if (threadIdx.x < 2 || hscale > 0.f) atomicMax(stat + threadIdx.x, v);
        }
        return;
    }
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const int64_t r = dst[j];
    if (r < 0) return;
    const float *src = rows + j * (int64_t)d;
    float *out = codes + r * (int64_t)d;
    const float inv = hscale > 0.f ? 1.f / hscale : 0.f;
    unsigned mabs = 0;
    float res = 0.f;
    for (int e = lane; e < d; e += 64) {
        const float x = src[e];
        out[e] = x;
        mabs = max(mabs, __float_as_uint(x) & 0x7fffffffu);
        if (hscale > 0.f) {
            const float q = x - mh_val(mh_half_bits(x * hscale)) * inv;
            res = fmaf(q, q, res);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mabs = max(mabs, (unsigned)__shfl_xor((int)mabs, o));
        res += __shfl_xor(res, o);
    }
    if (lane == 0) {
        ids[r] = ids_in[j];
        if (xnorm) xnorm[r] = norms[j];
        if (!stat) return;
        atomicMax(stat + 0, __float_as_uint(norms[j]));
        atomicMax(stat + 1, mabs);
        if (hscale > 0.f) atomicMax(stat + 2, __float_as_uint(res));
    }
}

// The batch's queries, one wave per query: t = 2^(14 − e_q), q·t split into two fp16 terms in the
// image's k-slot order, qsplit [query][term][super-step][g][8 halves]; its[q] = 1/(t·s) (a power of
// two), qres[q] = ‖q − (h + l)/t‖ and qres[nq + q] = ‖q − h/t‖ (×1.0001 for the fp32 sum; 2·nq floats).  A query whose scale leaves the safe
// range (non-finite entries, |e_q| > 100, 1/(t·s) not a normal float) gets zero terms and qres = +inf:
// the rerank flags it and it re-runs on the device in the direct form.
// qn (optional): also ‖q‖², in exactly row_norms_f32's order (vec4: float4 j = lane, lane + 64, …, four fmas
// each; else element-strided), so the coarse quantizer and the scan read the same bits they read before — the
// batch's query preparation in one launch.
__global__ void __launch_bounds__(256) ivf_split_queries_h(const float *__restrict__ Q, int64_t nq, int d, int nsup,
                                                           int es, uint4 *__restrict__ out, float *__restrict__ its,
                                                           float *__restrict__ qres, float *__restrict__ qn, int vec4) {
    // vec4 rows of ≤ 1024 dims: one load round trip for the row (≤ 4 float4 per lane), staged in LDS for the
    // split's k-slot order; ‖q‖² and the max come from the same registers (‖q‖² in row_norms_f32's order)
    __shared__ __attribute__((aligned(16))) float srow[4][1024];
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float *src = Q + q * (int64_t)d;
    unsigned mb = 0;
    if (vec4 && d <= 1024) {
        const float4 *p4 = reinterpret_cast<const float4 *>(src);
        const int n4 = d >> 2;
        float4 r4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = lane + 64 * i;
            r4[i] = j < n4 ? p4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 v = r4[i];
            if (lane + 64 * i < n4) {
                s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
                reinterpret_cast<float4 *>(srow[wv])[lane + 64 * i] = v;
            }
            mb = max(mb, max(max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu),
                             max(__float_as_uint(v.z) & 0x7fffffffu, __float_as_uint(v.w) & 0x7fffffffu)));
        }
        if (qn) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if (lane == 0) qn[q] = s;
        }
        __builtin_amdgcn_wave_barrier();
        src = srow[wv];
    } else {
        if (qn) {
            float s = 0.f;
            if (vec4) {
                const float4 *p4 = reinterpret_cast<const float4 *>(src);
                for (int j = lane; j < (d >> 2); j += 64) {
                    const float4 v = p4[j];
                    s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
                }
            } else {
                for (int j = lane; j < d; j += 64) s = fmaf(src[j], src[j], s);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
            if (lane == 0) qn[q] = s;
        }
        for (int e = lane; e < d; e += 64) mb = max(mb, __float_as_uint(src[e]) & 0x7fffffffu);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
    int eq = 0;
    if (mb != 0 && mb < 0x7f800000u) (void)frexpf(__uint_as_float(mb), &eq);
    const int et = 14 - eq;
    const int eits = -(et + es);
    const bool ok = mb < 0x7f800000u && eq >= -100 && eq <= 100 && eits >= -120 && eits <= 120;
    const float t = ldexpf(1.f, ok ? et : 0), inv_t = ldexpf(1.f, ok ? -et : 0);
    float r2 = 0.f, r1 = 0.f;  // two-term and one-term (high term only) split residuals
    for (int w = lane; w < nsup * 4; w += 64) {
        const int S = w >> 2, gg = w & 3;
        const int d0 = 32 * S + 4 * gg, d1 = d0 + 16;
        float a[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[j] = ok && d0 + j < d ? src[d0 + j] * t : 0.f;
            a[4 + j] = ok && d1 + j < d ? src[d1 + j] * t : 0.f;
        }
        unsigned hw[4], lw[4];
#pragma unroll
        for (int pr = 0; pr < 4; ++pr) {
            const float x0 = a[2 * pr], x1 = a[2 * pr + 1];
            hw[pr] = mh_pack(x0, x1);
            const float m0 = x0 - mh_val((unsigned short)(hw[pr] & 0xffffu)), m1 = x1 - mh_val((unsigned short)(hw[pr] >> 16));
            lw[pr] = mh_pack(m0, m1);
            r1 = fmaf(m0 * inv_t, m0 * inv_t, r1);
            r1 = fmaf(m1 * inv_t, m1 * inv_t, r1);
            const float e0 = (m0 - mh_val((unsigned short)(lw[pr] & 0xffffu))) * inv_t;
            const float e1 = (m1 - mh_val((unsigned short)(lw[pr] >> 16))) * inv_t;
            r2 = fmaf(e0, e0, r2);
            r2 = fmaf(e1, e1, r2);
        }
        out[((q * 2 + 0) * nsup + S) * 4 + gg] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        out[((q * 2 + 1) * nsup + S) * 4 + gg] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        r2 += __shfl_xor(r2, o);
        r1 += __shfl_xor(r1, o);
    }
    if (lane == 0) {
        its[q] = ldexpf(1.f, ok ? eits : 0);
        qres[q] = ok ? sqrtf(r2) * 1.0001f : __builtin_inff();
        qres[nq + q] = ok ? sqrtf(r1) * 1.0001f : __builtin_inff();  // a wide item's scan copies it over qres[q]
    }
}

template <int QT, bool IP, int NT, bool I8 = false>
__device__ __forceinline__ void mh_item(int d, const uint4 *__restrict__ codes_h, int64_t tp0,
                                        const float *__restrict__ xn, int64_t r0, int64_t r1, int nqi,
                                        const unsigned *__restrict__ qs, int stride, const float (&qn)[QT][4],
                                        const float (&qits)[QT][4], const unsigned (&qb)[QT][4],
                                        const float2 *__restrict__ qpar,
                                        const int *__restrict__ bucket, int boff, int nprobe,
                                        const int *__restrict__ slot_off, int chunk, int k, int sub, float *smem,
                                        unsigned *__restrict__ qbound, float *__restrict__ part_d,
                                        int *__restrict__ part_i, unsigned *prog, unsigned epoch, unsigned pword,
                                        const float *__restrict__ xs8) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = lane & 15, g = lane >> 4;
    const int nsup = I8 ? mi_nsup(d) : mh_nsup(d);  // (I8: 64-dim super-steps of the int8 image)
    const int npass_all = (int)ceil_div(r1 - r0, MF_PASS);
    const int npass = npass_all > wave ? (npass_all - wave + MF_WAVES - 1) / MF_WAVES : 0;
    // Round rotation (prog): the query groups of one chunk run as consecutive items on one XCD, each streaming the
    // whole chunk; an item that starts while another group of the chunk is under way begins at the round (8 passes)
    // that item last published and wraps around, so both read the same rows at about the same time and the later
    // one's reads hit the XCD's L2.  The slot's k-list does not depend on the order its rows are seen.
    int rr0 = 0;  // (pword: the chunk's progress word, loaded by the kernel ahead of the query fill)
    if (HIPANN_MH_FOLLOW && prog && npass > 0 && (pword >> 8) == (epoch & 0xffffffu)) rr0 = (int)(pword & 0xffu) % npass;
    auto rot = [&](int i) {  // i < npass
        if constexpr (!HIPANN_MH_FOLLOW) return i;
        const int r = i + rr0;
        return r < npass ? r : r - npass;
    };

    // per query: the sorted list (key, row) and the admission gate = the key of its k-th entry (a 16-row batch
    // merges when some lane's key is ≤ the gate: a superset of the lexicographic test, the merge itself is exact)
    uint64_t lst[QT][4];
    unsigned thr[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint64_t b = ((uint64_t)qb[qt][v] << 32) | MF_PAD_ID;
            lst[qt][v] = m < k ? b : MF_EMPTY;
            thr[qt][v] = qb[qt][v];
        }

    auto row_of = [&](int i, int r) -> int64_t {
        const int64_t row = r0 + (int64_t)(wave + MF_WAVES * rot(i)) * MF_PASS + 16 * r + m;
        return row < r1 ? row : r1 - 1;
    };
    const int ilast = npass > 0 ? npass - 1 : 0;
    const uint4 *rp;
    int ld_i = 0, ld_s = 0;  // stream position (super-steps), wave-uniform
    auto set_pass = [&](int i) { rp = codes_h + ((tp0 + wave + MF_WAVES * rot(i)) * nsup) * (MF_RT * 64) + lane; };
    // unconditional loads (past the wave's last step they re-read it): see mf_item
    auto next_load = [&](uint4 (&dst)[MF_RT]) {
        const int s = ld_i <= ilast ? ld_s : nsup - 1;
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) {
            if (HIPANN_MH_NT) {
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rp + (int64_t)s * (MF_RT * 64) + r * 64));
                dst[r] = make_uint4(v[0], v[1], v[2], v[3]);
            }
            else dst[r] = rp[(int64_t)s * (MF_RT * 64) + r * 64];
        }
        if (++ld_s == nsup) {
            ld_s = 0;
            ++ld_i;
            set_pass(ld_i <= ilast ? ld_i : ilast);
        }
    };

    uint4 ring[MH_P][MF_RT];
    float xnr[MF_RT] = {0.f, 0.f}, xsr[MF_RT] = {0.f, 0.f};  // (I8: the rows' scales)
    if (npass > 0) {
        set_pass(0);
#pragma unroll
        for (int p = 0; p < MH_P; ++p) next_load(ring[p]);
        if (!IP) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr[r] = xn[row_of(0, r)];
        }
        if constexpr (I8) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xsr[r] = xs8[row_of(0, r)];
        }
    }
    // the item's query image (and the wide items' parameters) were written by every thread before the call: wait for
    // them only now, with this wave's first MH_P super-steps of rows already in flight
    // (an LDS-only wait and the barrier: __syncthreads()'s fence would also drain the row loads, vmcnt(0))
    if (HIPANN_MH_EARLY) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const unsigned *qrow[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) qrow[qt] = qs + (qt * 16 + m) * stride + 4 * g;

    mf_f32x4 acc[QT][MF_RT];
    mf_i32x4 acci[QT][MF_RT];  // (I8: int32 sums)
    for (int i = 0; i < npass; ++i) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) {
                if constexpr (I8) acci[qt][r] = mf_i32x4{0, 0, 0, 0};
                else acc[qt][r] = mf_f32x4{0.f, 0.f, 0.f, 0.f};
            }
        float xnr_next[MF_RT] = {0.f, 0.f}, xsr_next[MF_RT] = {0.f, 0.f};
        if (!IP) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xnr_next[r] = xn[row_of(i + 1 <= ilast ? i + 1 : ilast, r)];
        }
        if constexpr (I8) {
#pragma unroll
            for (int r = 0; r < MF_RT; ++r) xsr_next[r] = xs8[row_of(i + 1 <= ilast ? i + 1 : ilast, r)];
        }
        for (int S0 = 0; S0 < nsup; S0 += MH_P) {
#pragma unroll
            for (int p = 0; p < MH_P; ++p) {
                const int S = S0 + p;
                uint4 qa[QT][NT];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                    for (int j = 0; j < NT; ++j) qa[qt][j] = *reinterpret_cast<const uint4 *>(qrow[qt] + (j * nsup + S) * 16);
                // the small query term first in every accumulator chain
#pragma unroll
                for (int j = NT - 1; j >= 0; --j)
#pragma unroll
                    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                        for (int r = 0; r < MF_RT; ++r) {
                            if constexpr (I8)
                                acci[qt][r] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(mf_i32x4, qa[qt][j]),
                                                                                   __builtin_bit_cast(mf_i32x4, ring[p][r]),
                                                                                   acci[qt][r], 0, 0, 0);
                            else acc[qt][r] = mh_mfma(qa[qt][j], ring[p][r], acc[qt][r]);
                        }
                next_load(ring[p]);
            }
        }
        const int64_t prow0 = r0 + (int64_t)(wave + MF_WAVES * rot(i)) * MF_PASS;
        // publish the round this item reaches next (wave 0; a later group of the chunk starts there)
        if (HIPANN_MH_FOLLOW && prog && wave == 0 && lane == 0)
            __hip_atomic_store(prog, (epoch << 8) | (unsigned)((rot(i) + 1) % npass), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) {
            const int64_t row = prow0 + 16 * r + m;
            const bool rok = row < r1;
            const unsigned rid = rok ? (unsigned)row : MF_PAD_ID;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    float qnv, qiv;
                    if constexpr (NT == 1) {  // wide items: (‖q‖², 1/(t·s)) from LDS (registers for 96 queries spill)
                        const float2 p = qpar[qt * 16 + 4 * g + v];
                        qnv = p.x;
                        qiv = p.y;
                    } else {
                        qnv = qn[qt][v];
                        qiv = qits[qt][v];
                    }
                    float key;
                    // I8: the sum as a whole-vector convert (per-element extracts of a bit-cast i32 MFMA result were
                    // miscompiled in the Flat int8 kernel), scaled by s_q·s_x
                    const float av = I8 ? __builtin_convertvector(acci[qt][r], mf_f32x4)[v] : acc[qt][r][v];
                    const float sc = I8 ? qiv * xsr[r] : qiv;
                    if (IP) {
                        key = -av * sc;
                    } else {
                        key = fmaf(-2.f * sc, av, qnv + xnr[r]);
                        key = key < 0.f ? 0.f : key;
                    }
                    const bool ok = rok && qt * 16 + 4 * g + v < nqi;
                    const unsigned ks = mf_sortable(key);
                    uint64_t cp = ok ? (((uint64_t)ks << 32) | rid) : MF_EMPTY;
                    if (__ballot(ok && ks <= thr[qt][v])) {
                        row_sort16(cp, m);
                        row_merge16(lst[qt][v], cp, m);
                        thr[qt][v] = row_kth_key(lst[qt][v], k - 1, g);
                    }
                }
        }
#pragma unroll
        for (int r = 0; r < MF_RT; ++r) {
            xnr[r] = xnr_next[r];
            xsr[r] = xsr_next[r];
        }
    }

    mf_finish_item<QT>(lst, smem, nqi, bucket, boff, nprobe, slot_off, chunk, k, sub, qbound, part_d, part_i);
}

// Copy the item's queries' first NT fp16 terms (of the TS in qsplit [query][term][S][g][4 dwords]: 2, or 1 for the
// int8 units) into LDS [query][term][S][g][4].
template <int NT, int TS = 2>
__device__ __forceinline__ void mh_fill(unsigned *qs, const uint4 *__restrict__ qsplit, int nsup, int stride, int nqi,
                                        const int *__restrict__ bucket, int boff, int nprobe) {
    const int per_q = NT * nsup * 4;
    for (int t = threadIdx.x; t < nqi * per_q; t += MF_THREADS) {
        const int q = t / per_q, rr = t - q * per_q;
        const int j = rr / (nsup * 4), r2 = rr - j * (nsup * 4);
        const int gq = bucket[boff + q] / nprobe;
        *reinterpret_cast<uint4 *>(qs + q * stride + r2 * 4 + j * nsup * 16) = qsplit[((int64_t)gq * TS + j) * nsup * 4 + r2];
    }
}

// ---- GEMM items --------------------------------------------------------------------------------------------------
// A list probed by more queries than a wide item holds (96 one-term queries fill the LDS) is scanned in items of up to
// MG_Q = 256 of them, shaped as a small GEMM: per 32-dim K-step the block stages, by LDS-DMA, the step's slice of 128
// database rows (4 passes × 2 row tiles × 1 KiB, straight from the tiled fp16 image) and of its 256 queries' high terms
// (16 pieces of 16 queries × 64 B, gathered per lane from the batch's query image), four stages deep (three K-steps in
// flight); wave (wr, wq) multiplies its 64 rows by its 64 queries (4 × 4 tiles of v_mfma_f32_16x16x32_f16) and keeps
// the same 16-lane DPP-row lists as the wide items for its queries.  A 2048-row chunk is 16 block steps; the list is
// streamed ceil(c / 256) times instead of ceil(c / 96).  LDS per K-step and wave: 4 + 4 ds_read_b128 for 16 MFMAs.
// The stored query slice is swizzled (group g of query q at unit 4q + (g ^ F(q)), F(q) = −((q >> 2) & 3) & 3) so that
// a wave's 16-query fragment read is conflict-free; the DMA lane that fills unit u loads the group that belongs there.
typedef __attribute__((address_space(3))) void mg_lds_void;
constexpr int MG_PASSES = 4;                        // 32-row passes per block step (128 rows)
constexpr int MG_NST = 4;                           // LDS stages
constexpr int MG_ROWU = MG_PASSES * MF_RT * 64;     // 16-B units of a stage's rows (8 KiB)
constexpr int MG_STU = MG_ROWU + MG_Q * 4;          // + the queries' slice (16 KiB)
constexpr size_t MG_XN = (size_t)MG_NST * MG_STU * 16;               // ‖x‖² of a block step's rows, by block parity
constexpr size_t MG_QPAR = MG_XN + 2 * MG_PASSES * MF_PASS * sizeof(float);  // (‖q‖², 1/(t·s)) per query
constexpr size_t MG_SCR = MG_QPAR + (size_t)MG_Q * sizeof(float2);  // the row halves' list merge
constexpr size_t MG_LDS = MG_SCR + (size_t)4 * 4 * 4 * 64 * sizeof(uint64_t);
static_assert(MG_LDS <= MF_LDS_MAX, "GEMM item LDS");
static_assert(MF_WAVES == 8, "GEMM items: 2 row halves x 4 query quarters");

template <bool IP>
__device__ __forceinline__ void mg_item(int d, const uint4 *__restrict__ codes_h, int64_t tp0, const float *xn, int64_t r0,
                                        int64_t r1, int nqi, const uint4 *__restrict__ qsplit, const float2 *qpar,
                                        const int *__restrict__ bucket, int boff, int nprobe,
                                        const int *__restrict__ slot_off, int chunk, int k, int sub, uint4 *stg,
                                        uint64_t *scr, unsigned *__restrict__ qbound, float *__restrict__ part_d,
                                        int *__restrict__ part_i) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m = lane & 15, g = lane >> 4;
    const int wr = wave & 1, wq = wave >> 1;  // row half (64 rows of a block step), query quarter (64 queries)
    const int nsup = mh_nsup(d);
    const int npass = (int)ceil_div(r1 - r0, MF_PASS);
    const int G = (int)ceil_div(npass, MG_PASSES) * nsup;  // K-steps of the item
    const int q0w = wq * 64;
    const int nqt_w = nqi > q0w ? min(4, (nqi - q0w + 15) >> 4) : 0;  // the wave's tiles holding a real query

    uint64_t lst[4][4];
    unsigned thr[4][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int q = q0w + qt * 16 + 4 * g + v;
            const unsigned qb = q < nqi ? __atomic_load_n(qbound + bucket[boff + q] / nprobe, __ATOMIC_RELAXED)
                                        : 0xffffffffu;
            lst[qt][v] = m < k ? (((uint64_t)qb << 32) | MF_PAD_ID) : MF_EMPTY;
            thr[qt][v] = qb;
        }

    // the wave's DMA pieces per K-step: row piece (pass wave >> 1, tile wave & 1) and query pieces 2·wave, 2·wave + 1
    const int rp_p = wave >> 1, rp_r = wave & 1;
    const uint4 *qsrc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ql = 16 * (2 * wave + i) + (lane >> 2);
        const int gq = bucket[boff + (ql < nqi ? ql : 0)] / nprobe;
        const int gs = (lane & 3) ^ ((-(lane >> 4)) & 3);  // the source group stored at this lane's unit
        qsrc[i] = qsplit + (int64_t)gq * 2 * nsup * 4 + gs;
    }
    // a block step's first K-step also brings its rows' ‖x‖² (L2): one dword DMA per wave, rows 64·(wave & 1) + lane of
    // the step into the parity-(blk & 1) buffer (the other waves repeat the two halves: every wave issues the same ops)
    float *xnb = reinterpret_cast<float *>(reinterpret_cast<char *>(stg) + MG_XN);
    auto issue = [&](int gk) {  // K-step min(gk, G − 1) into stage gk % MG_NST (past the end: a stage never read)
        const int gs = gk < G ? gk : G - 1;
        const int blk = gs / nsup, S = gs - blk * nsup;
        int pass = blk * MG_PASSES + rp_p;
        pass = pass < npass ? pass : npass - 1;
        uint4 *dst = stg + (gk % MG_NST) * MG_STU;
        if (!IP && S == 0) {
            const int64_t row = r0 + (int64_t)blk * (MG_PASSES * MF_PASS) + 64 * (wave & 1) + lane;
            __builtin_amdgcn_global_load_lds((const void *)(xn + (row < r1 ? row : r1 - 1)),
                                             (mg_lds_void *)(xnb + (blk & 1) * (MG_PASSES * MF_PASS) + 64 * (wave & 1)),
                                             4, 0, 0);
        }
        __builtin_amdgcn_global_load_lds(
            (const void *)(codes_h + ((tp0 + pass) * nsup + S) * (MF_RT * 64) + rp_r * 64 + lane),
            (mg_lds_void *)(dst + (rp_p * MF_RT + rp_r) * 64), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void *)(qsrc[i] + S * 4),
                                             (mg_lds_void *)(dst + MG_ROWU + (2 * wave + i) * 64), 16, 0, 0);
    };
    // waits (vmcnt: loads retire in issue order): at K-step gk the stage of gk must have landed; younger are the two
    // next K-steps' DMA ops — 3 each, 4 for a block step's first K-step (L2: its ‖x‖²)
    auto first_of_blk = [&](int x) { const int gs = x < G ? x : G - 1; return !IP && gs % nsup == 0; };

    if (G > 0) {
        issue(0);
        issue(1);
        issue(2);
    }
    mf_f32x4 acc[4][4];
    float xr[4] = {0.f, 0.f, 0.f, 0.f};
    int blk = 0, S = 0;
    const int fq = (-(m >> 2)) & 3;  // the swizzle of this lane's query rows
    for (int gk = 0; gk < G; ++gk) {
        if (S == 0)
#pragma unroll
            for (int qt = 0; qt < 4; ++qt)
#pragma unroll
                for (int rt = 0; rt < 4; ++rt) acc[qt][rt] = mf_f32x4{0.f, 0.f, 0.f, 0.f};
        const int younger = (int)first_of_blk(gk + 1) + (int)first_of_blk(gk + 2);  // wave-uniform
        if (younger == 0) __builtin_amdgcn_s_waitcnt(0xF70u | 6u);
        else if (younger == 1) __builtin_amdgcn_s_waitcnt(0xF70u | 7u);
        else __builtin_amdgcn_s_waitcnt(0xF70u | 8u);
        __builtin_amdgcn_s_barrier();  // every wave's stage gk landed; every wave done reading stage gk − 1
        asm volatile("" ::: "memory");
        issue(gk + 3);
        const uint4 *sb = stg + (gk % MG_NST) * MG_STU;
        uint4 rb[4], qa[4];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) rb[rt] = sb[((2 * wr + (rt >> 1)) * MF_RT + (rt & 1)) * 64 + lane];
#pragma unroll
        for (int qt = 0; qt < 4; ++qt)
            if (qt < nqt_w) qa[qt] = sb[MG_ROWU + (q0w + qt * 16 + m) * 4 + (g ^ fq)];
#pragma unroll
        for (int qt = 0; qt < 4; ++qt)
            if (qt < nqt_w)
#pragma unroll
                for (int rt = 0; rt < 4; ++rt) acc[qt][rt] = mh_mfma(qa[qt], rb[rt], acc[qt][rt]);
        if (++S == nsup) {
            // epilogue of block step blk: the wave's 64 rows × its queries into the lists
            if (!IP)
#pragma unroll
                for (int rt = 0; rt < 4; ++rt) xr[rt] = xnb[(blk & 1) * (MG_PASSES * MF_PASS) + wr * 64 + rt * 16 + m];
#pragma unroll
            for (int rt = 0; rt < 4; ++rt) {
                const int64_t row = r0 + (int64_t)blk * (MG_PASSES * MF_PASS) + wr * 64 + rt * 16 + m;
                const bool rok = row < r1;
                const unsigned rid = rok ? (unsigned)row : MF_PAD_ID;
#pragma unroll
                for (int qt = 0; qt < 4; ++qt) {
                    if (qt >= nqt_w) continue;  // wave-uniform
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int q = q0w + qt * 16 + 4 * g + v;
                        const float2 p = qpar[q];
                        float key;
                        if (IP) {
                            key = -acc[qt][rt][v] * p.y;
                        } else {
                            key = fmaf(-2.f * p.y, acc[qt][rt][v], p.x + xr[rt]);
                            key = key < 0.f ? 0.f : key;
                        }
                        const bool ok = rok && q < nqi;
                        const unsigned ks = mf_sortable(key);
                        uint64_t cp = ok ? (((uint64_t)ks << 32) | rid) : MF_EMPTY;
                        if (__ballot(ok && ks <= thr[qt][v])) {
                            row_sort16(cp, m);
                            row_merge16(lst[qt][v], cp, m);
                            thr[qt][v] = row_kth_key(lst[qt][v], k - 1, g);
                        }
                    }
                }
            }
            S = 0;
            ++blk;
        }
    }
    // drain the DMA issued past the end before the LDS is reused or released
    __builtin_amdgcn_s_waitcnt(0xF70u);
    __syncthreads();
    if (!sub) {  // the two row halves' lists of each query quarter: wr = 1 hands its lists to wr = 0
        uint64_t *sw = scr + (size_t)wq * 4 * 4 * 64;
        if (wr == 1)
#pragma unroll
            for (int qt = 0; qt < 4; ++qt)
#pragma unroll
                for (int v = 0; v < 4; ++v) sw[(qt * 4 + v) * 64 + lane] = lst[qt][v];
        __syncthreads();
        if (wr == 0)
#pragma unroll
            for (int qt = 0; qt < 4; ++qt)
#pragma unroll
                for (int v = 0; v < 4; ++v) row_merge16(lst[qt][v], sw[(qt * 4 + v) * 64 + lane], m);
    }
    if ((sub || wr == 0) && m < k) {
#pragma unroll
        for (int qt = 0; qt < 4; ++qt)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int q = q0w + qt * 16 + 4 * g + v;
                if (q >= nqi) continue;
                const int pr = bucket[boff + q];
                const int64_t slot = (int64_t)slot_off[pr] + chunk;
                const uint64_t e = lst[qt][v];
                const unsigned id = (unsigned)e;
                const bool real = e != MF_EMPTY && id != MF_PAD_ID;
                const int64_t off = (sub ? slot * MF_WAVES + wr : slot) * k + m;
                part_d[off] = real ? mf_unsortable((unsigned)(e >> 32)) : __builtin_inff();
                part_i[off] = real ? (int)id : (int)MF_PAD_ID;
                if (m == k - 1 && real) atomicMin(qbound + pr / nprobe, (unsigned)(e >> 32));
                if (sub && wr == 0)  // the slot's other sub-lists (MF_WAVES per slot; two row halves here) stay empty
                    for (int s2 = 2; s2 < MF_WAVES; ++s2) {
                        part_d[(slot * MF_WAVES + s2) * k + m] = __builtin_inff();
                        part_i[(slot * MF_WAVES + s2) * k + m] = (int)MF_PAD_ID;
                    }
            }
    }
}

// I8: the int8 image (every item one-term: units in qsplit, s_q in its, s_x in xs8; no residual copy)
template <bool IP, bool I8>
__global__ void __launch_bounds__(MF_THREADS, MF_WAVES / 4)
ivf_scan_mfma_h(const uint4 *__restrict__ qsplit, const float *__restrict__ qnorm, const float *__restrict__ its, int d,
                const uint4 *__restrict__ codes_h, const int64_t *__restrict__ tpass_off, const float *__restrict__ xn,
                const int64_t *__restrict__ list_off, const int *__restrict__ list_len, const int *__restrict__ cnt, const int *__restrict__ bucket_off,
                const int *__restrict__ item_off, const int *__restrict__ bucket, const int *__restrict__ slot_off,
                int nlist, int nprobe, int group, int k, int sub, unsigned *__restrict__ qbound, float *__restrict__ part_d,
                int *__restrict__ part_i, float *__restrict__ qres, int nq, int remap, unsigned *__restrict__ prog,
                int nprog, unsigned epoch, const float *__restrict__ xs8) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int total = item_off[nlist];
    if ((int)blockIdx.x >= total) return;
    const int item = remap ? xcd_remap((int)blockIdx.x, total) : (int)blockIdx.x;
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int64_t lr0 = list_off[l], lr1 = lr0 + list_len[l];
    const int c = cnt[l];
    const int cls = ivf_list_class(c, group);  // block-uniform
    const bool wide = I8 || cls == 1;
    const int ng = ivf_ngroups(c, group);
    const int rem = item - item_off[l];
    const int chunk = rem / ng, grp = rem - chunk * ng;
    const int q_begin = (int)((int64_t)grp * c / ng), q_end = (int)((int64_t)(grp + 1) * c / ng);
    const int nqi = q_end - q_begin;
    const int64_t r0 = lr0 + (int64_t)chunk * MF_CH;
    const int64_t r1 = r0 + MF_CH < lr1 ? r0 + MF_CH : lr1;
    const int boff = bucket_off[l] + q_begin;
    const int nqt = (nqi + 15) >> 4;

    if (!I8 && cls == 2) {
        uint4 *stg = reinterpret_cast<uint4 *>(smem);
        float2 *gpar = reinterpret_cast<float2 *>(reinterpret_cast<char *>(smem) + MG_QPAR);
        for (int t = threadIdx.x; t < nqi; t += MF_THREADS) {
            const int qi = bucket[boff + t] / nprobe;
            gpar[t] = make_float2(IP ? 0.f : qnorm[qi], its[qi]);
            qres[qi] = qres[nq + qi];  // one-term scan keys: the rerank's bound takes the one-term residual
        }
        __syncthreads();
        const int64_t tpg = tpass_off[l] + (int64_t)chunk * (MF_CH / MF_PASS);
        mg_item<IP>(d, codes_h, tpg, xn, r0, r1, nqi, qsplit, gpar, bucket, boff, nprobe, slot_off, chunk, k, sub, stg,
                    reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(smem) + MG_SCR), qbound, part_d, part_i);
        return;
    }
    // the chunk's progress word, loaded before the query fill so that its latency hides behind it
    const int64_t tp0 = tpass_off[l] + (int64_t)chunk * (MF_CH / MF_PASS);
    unsigned *pw = HIPANN_MH_FOLLOW && prog && nprog > 0 ? prog + (int)((tp0 >> 6) % nprog) : nullptr;
    const unsigned pword = pw ? (unsigned)__builtin_amdgcn_readfirstlane(
                                    (int)__hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              : 0u;
    unsigned *qs = reinterpret_cast<unsigned *>(smem);
    const int nsup = I8 ? mi_nsup(d) : mh_nsup(d);
    const int stride = I8 ? mi_nsup(d) * 16 + 8 : mh_stride(d, wide ? 1 : 2);
    float2 *qpar = reinterpret_cast<float2 *>(qs + nqi * stride);  // wide items: (‖q‖², 1/(t·s)) after the image
    if (wide) {
        mh_fill<1, I8 ? 1 : 2>(qs, qsplit, nsup, stride, nqi, bucket, boff, nprobe);
        for (int t = threadIdx.x; t < nqi; t += MF_THREADS) {
            const int qi = bucket[boff + t] / nprobe;
            qpar[t] = make_float2(IP ? 0.f : qnorm[qi], its[qi]);
            // these queries' scan keys miss the low term: the rerank bounds them with the one-term residual (every
            // item of the query's wide lists writes the same value)
            if (!I8) qres[qi] = qres[nq + qi];
        }
    } else if constexpr (!I8) {
        mh_fill<2>(qs, qsplit, nsup, stride, nqi, bucket, boff, nprobe);
    }
    if (!HIPANN_MH_EARLY) __syncthreads();  // (early: mh_item waits for the fill after issuing its first row loads)

    const int lane = threadIdx.x & 63, g = lane >> 4;
#define MH_ARGS d, codes_h, tp0, xn, r0, r1, nqi, qs, stride, qn, qi_s, qb, qpar, bucket, boff, nprobe, slot_off, chunk, k, sub, smem, \
                qbound, part_d, part_i, pw, epoch, pword, xs8
#define MH_QN(QTV)                                                                                          \
    float qn[QTV][4], qi_s[QTV][4];                                                                         \
    unsigned qb[QTV][4];                                                                                    \
    _Pragma("unroll") for (int qt = 0; qt < QTV; ++qt) _Pragma("unroll") for (int v = 0; v < 4; ++v) {      \
        const int q = qt * 16 + 4 * g + v;                                                                  \
        const int qi = q < nqi ? bucket[boff + q] / nprobe : 0;                                             \
        qn[qt][v] = (!IP && !wide && q < nqi) ? qnorm[qi] : 0.f;                                            \
        qi_s[qt][v] = !wide && q < nqi ? its[qi] : 0.f;                                                     \
        qb[qt][v] = q < nqi ? __atomic_load_n(qbound + qi, __ATOMIC_RELAXED) : 0xffffffffu;                 \
    }
#define MH_CASE(QTV, NTV) { MH_QN(QTV) mh_item<QTV, IP, NTV, I8>(MH_ARGS); }
    if (wide) {
        // nqi > narrow / 2 (a wide list has more than one narrow group of queries, split evenly) unless every list
        // is wide (narrow 0, A/B)
        if (nqt <= 1) MH_CASE(1, 1)
        else if (nqt == 2) MH_CASE(2, 1)
        else if (nqt == 3) MH_CASE(3, 1)
        else if (nqt == 4) MH_CASE(4, 1)
        else if (nqt == 5) MH_CASE(5, 1)
        else MH_CASE(6, 1)
    } else if constexpr (!I8) {
        if (nqt <= 1) MH_CASE(1, 2)
        else if (nqt == 2) MH_CASE(2, 2)
        else MH_CASE(3, 2)
    }
#undef MH_CASE
#undef MH_QN
#undef MH_ARGS
}

int ivf_mfma_h_group(int d) { return mh_group_packed(d); }
int ivf_scan_sublists() { return MF_WAVES; }
int64_t ivf_half_pass_bytes(int d) { return (int64_t)mh_nsup(d) * MF_RT * 64 * 16; }
int64_t ivf_half_qsplit_bytes(int64_t nq, int d) { return nq * 2 * mh_nsup(d) * 64; }
bool ivf_mfma_h_supported(int d, int k) { return d >= 1 && k >= 1 && k <= MF_KMAX && mh_group(d) >= 16; }
// int8 image: every item one-term, up to 96 queries (MH_QTW tiles) that fit the LDS with their (‖q‖², s_q)
int ivf_mfma_i8_group(int d) {
    const int g = (int)(MF_LDS_MAX / ((size_t)(mi_nsup(d) * 16 + 8) * 4 + 8)) / 16 * 16;
    return (g < 16 * MH_QTW ? g : 16 * MH_QTW) << 8;
}
int64_t ivf_i8_pass_bytes(int d) { return (int64_t)mi_nsup(d) * MF_RT * 64 * 16; }
int64_t ivf_i8_qimg_bytes(int64_t nq, int d) { return nq * mi_nsup(d) * 64; }
bool ivf_mfma_i8_supported(int d, int k) {
    return d >= 1 && k >= 1 && k <= MF_KMAX && ivf_group_wide(ivf_mfma_i8_group(d)) >= 16;
}
void launch_ivf_tile_i8(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                        int nlist, int64_t total_pass, int d, void *dst, float *xs8, hipStream_t st,
                        const int64_t *pass_ids) {
    if (total_pass <= 0) return;
    HIPANN_REQUIRE(total_pass < (int64_t)0x7fffffff, "too many passes");
    hipLaunchKernelGGL(ivf_tile_i8, dim3((unsigned)total_pass), dim3(256), 0, st, codes, list_off, list_len, tpass_off,
                       nlist, d, mi_nsup(d), static_cast<uint4 *>(dst), xs8, pass_ids);
    HIPANN_CHECK(hipGetLastError());
}
void launch_ivf_i8_residual(const float *codes, int64_t n, int d, unsigned *out, hipStream_t st) {
    HIPANN_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned), st));
    if (n <= 0) return;
    HIPANN_REQUIRE(ceil_div(n, 4) < (int64_t)0x7fffffff, "too many rows");
    hipLaunchKernelGGL(ivf_i8_residual, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, codes, n, d, out);
    HIPANN_CHECK(hipGetLastError());
}
void launch_ivf_split_queries_i8(const float *Q, int64_t nq, int d, void *qi8, float *qs8, float *qres8,
                                 hipStream_t st) {
    if (nq <= 0) return;
    HIPANN_REQUIRE(ceil_div(nq, 4) < (int64_t)0x7fffffff, "too many queries");
    hipLaunchKernelGGL(ivf_split_queries_i8, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, Q, nq, d, mi_nsup(d),
                       static_cast<uint4 *>(qi8), qs8, qres8);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_max_abs(const float *x, int64_t cnt, unsigned *out, hipStream_t st) {
    HIPANN_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned), st));
    if (cnt <= 0) return;
    const unsigned blocks = (unsigned)std::min<int64_t>(4096, ceil_div(cnt, 256));
    hipLaunchKernelGGL(ivf_max_abs, dim3(blocks), dim3(256), 0, st, x, cnt, out);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_tile_half(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                          int nlist, int64_t total_pass, int d, float scale, void *dst, hipStream_t st,
                          const int64_t *pass_ids) {
    if (total_pass <= 0) return;
    HIPANN_REQUIRE(total_pass < (int64_t)0x7fffffff, "too many passes");
    hipLaunchKernelGGL(ivf_tile_half, dim3((unsigned)total_pass), dim3(256), 0, st, codes, list_off, list_len, tpass_off,
                       nlist, d, mh_nsup(d), scale, static_cast<uint4 *>(dst), pass_ids);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_half_residual(const float *codes, int64_t n, int d, float scale, unsigned *out, hipStream_t st) {
    HIPANN_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned), st));
    if (n <= 0) return;
    HIPANN_REQUIRE(ceil_div(n, 4) < (int64_t)0x7fffffff, "too many rows");
    hipLaunchKernelGGL(ivf_half_residual, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, codes, n, d, scale,
                       1.f / scale, out);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_append_rows(const float *rows, const float *norms, const int64_t *dst, const int64_t *ids_in, int64_t n,
                            int d, float *codes, int64_t *ids, float *xnorm, const int *newlen, int *list_len, int nlist,
                            float hscale, unsigned *stat, hipStream_t st) {
    int64_t blocks = std::max(ceil_div(n, (int64_t)4), ceil_div((int64_t)nlist, (int64_t)256));
    if (!dst) blocks = std::min<int64_t>(blocks, 64);  // statistics only: a grid-stride loop, one atomic per block
    HIPANN_REQUIRE(blocks < (int64_t)0x7fffffff, "append block too large");
    if (stat) HIPANN_CHECK(hipMemsetAsync(stat, 0, sizeof(unsigned) * 4, st));
    hipLaunchKernelGGL(ivf_append_rows, dim3((unsigned)blocks), dim3(256), 0, st, rows, norms, dst, ids_in, n, d, codes,
                       ids, xnorm, newlen, list_len, nlist, hscale, stat);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_split_queries_h(const float *Q, int64_t nq, int d, int es, void *qsplit, float *its, float *qres,
                                float *qn, hipStream_t st) {
    if (nq <= 0) return;
    const int vec4 = (d % 4 == 0) && ((uintptr_t)Q % 16 == 0);  // launch_row_norms' rule
    hipLaunchKernelGGL(ivf_split_queries_h, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, Q, nq, d, mh_nsup(d), es,
                       static_cast<uint4 *>(qsplit), its, qres, qn, vec4);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_scan_mfma_h(const float *Q, int64_t nq, void *qsplit, float *its, float *qres, int es, const float *qn,
                            int d, int metric, const void *codes_h, const int64_t *tpass_off, const float *xn,
                            const int64_t *list_off, const int *list_len, const int *cnt, const int *bucket_off,
                            const int *item_off, const int *bucket, const int *slot_off, int nlist, int nprobe, int k,
                            int64_t max_items, unsigned *qbound, float *pd, int *pi, hipStream_t st, bool split_done,
                            int sub, unsigned *prog, int nprog, unsigned epoch, int i8mode, const float *xs8) {
    if (max_items <= 0 || nq <= 0) return;
    HIPANN_REQUIRE(max_items < (int64_t)0x7fffffff, "too many IVF work items");
    HIPANN_REQUIRE(qsplit && its && qres && codes_h, "fp16 IVF scan: missing buffers");
    HIPANN_REQUIRE(i8mode ? ivf_mfma_i8_supported(d, k) && xs8 && split_done : ivf_mfma_h_supported(d, k),
                   "fp16 / int8 IVF scan needs k <= 16 (int8: scales and prepared queries)");
    HIPANN_REQUIRE(metric == kIP || (qn && xn), "decomposed L2 scan needs query and row norms");
    const int nsup = mh_nsup(d);
    uint4 *qs = static_cast<uint4 *>(qsplit);
    if (!split_done)
        hipLaunchKernelGGL(ivf_split_queries_h, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, Q, nq, d, nsup, es, qs,
                           its, qres, nullptr, (d % 4 == 0) && ((uintptr_t)Q % 16 == 0));
    const int group = i8mode ? ivf_mfma_i8_group(d) : mh_group_packed(d);
    const int gw = ivf_group_wide(group);
    const size_t merge = (size_t)(MF_WAVES / 2) * (gw ? MH_QTW : MF_QTMAX) * 4 * 64 * sizeof(float2);
    const size_t wstride = i8mode ? (size_t)(mi_nsup(d) * 16 + 8) * 4 : (size_t)mh_stride(d, 1) * 4;
    const size_t smem = std::max({(size_t)ivf_group_narrow(group) * mh_stride(d) * 4, (size_t)gw * (wstride + 8), merge,
                                  ivf_group_gemm(group) ? MG_LDS : (size_t)0});
    HIPANN_REQUIRE(smem <= MF_LDS_MAX, "fp16 IVF scan: LDS image too large");
    HIPANN_REQUIRE(nq < (int64_t)0x7fffffff, "fp16 IVF scan: batch too large");
    dim3 grid((unsigned)max_items), block(MF_THREADS);
    const uint4 *ch = static_cast<const uint4 *>(codes_h);
    // HIPANN_IVF_REMAP=0 (A/B): consecutive items (a chunk's query groups) dealt round-robin over the XCDs instead of
    // contiguous runs per XCD
    static const int remap = [] { const char *e = std::getenv("HIPANN_IVF_REMAP"); return !e || std::atoi(e) ? 1 : 0; }();
#define MH_LAUNCH_ARGS qs, qn, its, d, ch, tpass_off, xn, list_off, list_len, cnt, bucket_off, item_off, bucket, slot_off, nlist, nprobe, \
                       group, k, sub, qbound, pd, pi, qres, (int)nq, remap, prog, nprog, epoch, xs8
    if (i8mode) {
        if (metric == kIP) hipLaunchKernelGGL((ivf_scan_mfma_h<true, true>), grid, block, smem, st, MH_LAUNCH_ARGS);
        else hipLaunchKernelGGL((ivf_scan_mfma_h<false, true>), grid, block, smem, st, MH_LAUNCH_ARGS);
    } else {
        if (metric == kIP) hipLaunchKernelGGL((ivf_scan_mfma_h<true, false>), grid, block, smem, st, MH_LAUNCH_ARGS);
        else hipLaunchKernelGGL((ivf_scan_mfma_h<false, false>), grid, block, smem, st, MH_LAUNCH_ARGS);
    }
#undef MH_LAUNCH_ARGS
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
