// flat_b16k64.hip — the Flat bf16 filter scan (form kFlatBf16Exact) of a bounded pass: 64-dim K-steps on
// v_mfma_f32_16x16x32_bf16, a 2-K-step-deep memory pipeline, and the passing rows appended to per-(query,
// split) candidate buffers in global memory instead of per-query top-k lists in LDS.
//
// Same keys and images as flat_bf16_topk (flat_bf16.hip: MetalIndexFlat::search's GEMM + select for nq >= 20,
// faiss-metal/src/MetalIndexFlat.mm:294-369): key = ‖q‖² + ‖x‖² − 2·q̂·x̂ (L2, clamped at 0) or −q̂·x̂ (IP) from
// one bf16 product per element, as the filter of the exact fp32 rerank (ivf_rerank_topk).  A pass runs under a
// per-query bound T (flat_bf16_seed on a sample, then flat_cand_bound on the previous pass's candidates): every
// row with key ≤ T is appended to its (query, split) buffer; flat_cand_select then keeps each query's k best.
//   * tile = 256 queries × 256 database rows, K-step = 64 dims (two 32-dim image chunks, consecutive in the
//     tiled image); wave w owns queries [32w, 32w+32) × all 256 rows = 2 × 16 accumulators of 16 × 16 (the
//     256² recipe of cdna_hip_programming.md §5 with the query operand in registers);
//   * memory: the database tile streams by LDS-DMA into 5 stages of 32 KB three K-steps ahead, the query
//     fragments into a 2-slot register ring one K-step ahead; loads retire in issue order under vmcnt, so each
//     K-step issues A(g+1) before B(g+3) and one counted vmcnt(4) keeps B(g+2), B(g+3) in flight.  Measured on
//     10M × 768 with 3 stages and one K-step in flight for both (timing ablations):
//     the compute + LDS structure alone runs at 0.74 of dense bf16; with one K-step in flight the tile DMA and
//     the fragment loads added 3.5 and 2.4 ms to its 8.5 ms;
//   * the lists left LDS (5 stages need all 160 KiB): with a bound from a sample the passing rows are few
//     (≈12 per query and split at 10M rows), so the epilogue appends them (one scattered store each, the count
//     in a register) — no LDS round trips, no sorting in the scan.
#include "runtime.hpp"
#include "wave_topk.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

namespace hipann {

typedef __bf16 k64_b16x8 __attribute__((ext_vector_type(8)));
typedef float k64_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned k64_u32x4 __attribute__((ext_vector_type(4)));
typedef int k64_i32x4 __attribute__((ext_vector_type(4)));
typedef float k64_f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void k64_lds_void;

// Tuning builds only (timing ablations, wrong results): bit 0 drops the database-tile DMA, bit 1 the query-fragment
// loads, bit 2 the epilogue's candidate filter, bit 3 the per-K-step barrier, bit 4 the filter's append path (the
// compare and ballot kept), bit 5 the per-query scales (one per tile), bit 6 the accumulator reset, bit 7 the whole
// epilogue (the accumulators xor-reduced and reset).  Product builds: 0.
#ifndef HIPANN_K64_ABLATE
#define HIPANN_K64_ABLATE 0
#endif
constexpr int K64_TN = 256;               // database rows per tile
constexpr int K64_QM = 256;               // queries per block (8 waves × 32, or 4 waves × 64)
constexpr int K64_NB = 5;                 // LDS stages: g read, g+1 .. g+3 landing / in flight
constexpr int K64_BU = K64_TN * 4;        // 16-B units of one 32-dim chunk of a database tile
constexpr int K64_SU = 2 * K64_BU;        // units per stage (one 64-dim K-step): 32 KB
constexpr size_t K64_LDS = (size_t)K64_NB * K64_SU * 16;
static_assert(K64_LDS <= 160 * 1024, "LDS");
// MBW = 16-query accumulator row blocks per wave: 2 → 8 waves of 32 queries (two waves per SIMD, 256 registers);
// 4 → 4 waves of 64 queries (one wave per SIMD, 512 registers: the accumulators in AGPRs), each B fragment read
// from LDS feeding four MFMAs instead of two — half the LDS reads and barrier arrivals per MFMA
template <int MBW> struct K64Geom {
    static constexpr int W = 16 / MBW;                 // waves per block
    static constexpr int PIECES = K64_SU / 64 / W;     // 1-KiB LDS-DMA pieces per wave per K-step
    static_assert(PIECES * 64 * W == K64_SU, "pieces split evenly");
};

// Epilogue of one tile for accumulator row (MB, I).  On entry sm[jb][i] = s = 2·q·x − ‖x‖² (L2; 2·q·x for IP;
// −inf past N) of the wave's query 16·MB + 4·(lane >> 4) + i and database row x0 + 16·jb + (lane & 15); a row
// passes its query's bound when s ≥ cth = ‖q‖² − T (L2) or −2·T (IP) — cthm[i] is the lane's own query's (its
// 16-lane group).  Passing rows (rare) are appended to the query's buffer with key = ‖q‖² − s
// (L2, clamped at 0) or −s/2 = −q·x (IP); cntv lane j holds the count of the wave's query j (it keeps
// counting past cap: flat_cand_select flags an overflowed query for the exact fallback).
template <bool L2M, int MB, int I, int NJ>
__device__ __forceinline__ void k64_epilogue_row(const k64_f32x4 (&sm)[NJ], float mxi, const float (&cthm)[4], float qnl,
                                                 int &cntv, int64_t x0, float *__restrict__ cand_d,
                                                 int *__restrict__ cand_i, int64_t cbase, int64_t cq, int cap,
                                                 int lane, int JB0) {
    // sm[j] = s of row block JB0 + j (one half of the tile's 16; the halves keep the epilogue's live registers to 32
    // values).  mxi = max over the lane's 8 rows of sm[·][I] (the caller's reduction): one compare for the 8 (NaN
    // never passes: fmaxf drops NaN operands, an all-NaN max compares false)
    const unsigned long long m = __ballot(mxi >= cthm[I]);
    if (m == 0ull) return;
    if constexpr ((HIPANN_K64_ABLATE & 16) != 0) {  // (tuning: the slow path's cost, not its work)
        cntv += __popcll(m);
        return;
    }
    // the lane's passing columns (bit j: row block JB0 + j)
    unsigned pm = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) pm |= sm[j][I] >= cthm[I] ? 1u << j : 0u;
#pragma unroll 1
    for (int fq = 0; fq < 4; ++fq) {
        unsigned grp = (unsigned)(m >> (16 * fq)) & 0xffffu;  // lanes of query fq holding a passing row
        if (grp == 0u) continue;
        const int qw = 16 * MB + 4 * fq + I;  // the query's index in the wave
        const float qnr = L2M ? readlane_f(qnl, qw) : 0.f;
        int c = readlane_i(cntv, qw);
        float *cd = cand_d + cbase + (int64_t)qw * cq;
        int *ci = cand_i + cbase + (int64_t)qw * cq;
        while (grp) {
            const int l = __ffs(grp) - 1;
            grp &= grp - 1;
            const int src = 16 * fq + l;
            unsigned pml = (unsigned)__builtin_amdgcn_readlane((int)pm, src);
            while (pml) {
                const int jl = __ffs(pml) - 1;
                pml &= pml - 1;
                const int jb = JB0 + jl;
                float sv = sm[0][I];
#pragma unroll
                for (int j = 1; j < NJ; ++j) sv = jl == j ? sm[j][I] : sv;
                sv = readlane_f(sv, src);
                float key;
                if (L2M) {
                    key = qnr - sv;
                    key = key < 0.f ? 0.f : key;
                } else {
                    key = -0.5f * sv;
                }
                if (lane == 0 && c < cap) {
                    cd[c] = key;
                    ci[c] = (int)(x0 + 16 * jb + l);
                }
                ++c;
            }
        }
        cntv = lane == qw ? c : cntv;
    }
}

// One bounded pass of a split: tiles [tile_begin, tile_end) of split `split` for the block's 256 queries.
// Candidate buffers: cand_[dn]{[(q·nsplit + split)·cap + j]}, counts cand_n[q·nsplit + split] (resume: the
// previous pass's count is continued).  bound[q]: the pass's T (k-th best key of a sample / previous pass,
// with margin, flat_keys_kth / flat_cand_bound).
// KEYS (the sample pass that seeds the bound): no filter, every key of the block's tiles goes to
// cand_d[q·N + row] (a dense nq × N key matrix over the N sample rows; bound, cand_i, cand_n unused).
// I8 (form kFlatI8Exact): the same tiles and schedule over an int8 image (a 16-B unit = 16 dims, so one 64-B
// chunk row covers 64 dims and a K-step 128) on v_mfma_i32_16x16x64_i8 — twice the dims per instruction and
// per byte moved.  The int32 sums are exact (|acc| <= d·127² < 2^24 for d <= 1040) and live in the float
// accumulators' registers bit for bit until the tile's epilogue turns them into q·x = acc·s_q·s_x with the
// per-query / per-row scales (qscale / xscale); everything after that is the bf16 path's.
// STAG (A/B only, HIPANN_K64_STAGGER=1; measured slower, see launch_flat_bf16_k64) (the int8 bounded passes,
// d ≥ 384): waves W/2..W−1 run half a K-step behind waves 0..W/2−1 — in K-step g's
// barrier interval a late wave computes chunk 1 of g − 1, then (when g − 1 ended a tile) its epilogue, then chunk 0 of
// g.  Waves w and w + W/2 share a SIMD, so one wave's epilogue (≈ 650 VALU instructions per tile) and LDS read burst
// run beside its partner's MFMAs instead of both waves converting at the same barrier-aligned moment
// (MI355X_MICROARCH.md, two waves per SIMD, item 9).  Same loads, same order, same counted waits, one extra barrier
// interval at the end; the stage a late wave still reads (g − 1) is never the one refilled in interval g ((g + 3) mod 5).
template <bool L2M, bool KEYS, bool I8 = false, int MBW = 2, bool STAG = false>
__global__ void __launch_bounds__(64 * K64Geom<MBW>::W, 1) __attribute__((amdgpu_waves_per_eu(1, 2)))
flat_bf16_k64(const k64_u32x4 *__restrict__ Qt, const float *__restrict__ qnorm, int64_t nq,
              const k64_u32x4 *__restrict__ Xt, const float *xnorm, int64_t N, int nk, int nqt, int nsplit,
              int64_t tiles_per_split, int64_t tile_begin, int64_t tile_end, const float *__restrict__ bound,
              float *__restrict__ cand_d, int *__restrict__ cand_i, int *__restrict__ cand_n, int cap,
              int resume, const float *__restrict__ qscale, const float *xscale) {
    constexpr int NB = K64_NB;
    constexpr int QW = 16 * MBW;  // queries per wave
    constexpr int PIECES = K64Geom<MBW>::PIECES;
    extern __shared__ __attribute__((aligned(16))) k64_u32x4 smem_k64[];

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * K64_QM;
    const int64_t ntiles = ceil_div(N, K64_TN);
    const int64_t ts = (int64_t)split * tiles_per_split;
    const int64_t t0 = ts + tile_begin;
    const int64_t te = ts + (tile_end < tiles_per_split ? tile_end : tiles_per_split);
    const int64_t t1 = te < ntiles ? te : ntiles;
    const int ns = nk >> 1;  // K-steps per tile (nk even)
    const int64_t G = t1 > t0 ? (t1 - t0) * ns : 0;

    const int tid = threadIdx.x;
    // wave-uniform (readfirstlane): the wave's bases and buffer pointers live in SGPRs, not VGPRs
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int m16 = lane & 15, g4 = lane >> 4;
    const int64_t q0w = q0 + QW * wave + 4 * g4;  // + 16·mb + i: the lane's accumulator query rows

    // per-lane state of the wave's QW queries (lane j: query QW·wave + j): ‖q‖², candidate count
    const int64_t qlane = q0 + QW * wave + (lane & (QW - 1));
    float qnl = 0.f;
    if (L2M) qnl = qlane < nq ? qnorm[qlane] : 0.f;
    int cntv = 0;
    if (!KEYS && resume && lane < QW && qlane < nq) cntv = cand_n[qlane * nsplit + split];
    float cth[MBW][4];
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t q = q0w + 16 * mb + i;
            const float qn = (L2M && q < nq) ? qnorm[q] : 0.f;
            if constexpr (KEYS) {
                cth[mb][i] = qn;  // the keys pass keeps ‖q‖² of the lane's rows here
            } else {
                const float thr = q < nq ? bound[q] : -__builtin_inff();  // −inf: rows past nq pass nothing
                cth[mb][i] = L2M ? qn - thr : -2.f * thr;
            }
        }
    // int8: 2·s_q of the lane's accumulator query rows (the 2 of s = 2·q·x − ‖x‖² folded in)
    float csq[MBW][4];
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t q = q0w + 16 * mb + i;
            csq[mb][i] = I8 && q < nq ? 2.f * qscale[q] : 2.f;
        }
    const int64_t cq = (int64_t)nsplit * cap;  // buffer stride between consecutive queries
    const int64_t cbase = ((q0 + QW * wave) * nsplit + split) * (int64_t)cap;

    // K-step g = (t − t0)·ns + s covers image chunks 2s, 2s + 1 of tile t: 2·K64_BU consecutive units
    const k64_u32x4 *Xb = Xt + t0 * nk * K64_BU + lane;
    // the lane's query fragments: rows QW·wave + 16·mb + m16, unit c = g4 of each 32-dim chunk
    const k64_u32x4 *Qw = Qt + (int64_t)qt * nk * (K64_QM * 4) + g4 * K64_QM;
    int qrow[MBW];
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb) qrow[mb] = (QW * wave + 16 * mb + m16) ^ (g4 << 1);
    // query fragments: a 3-slot register ring (K-step g+2's loaded while g is computed); the loop is unrolled by
    // three so the slot is a compile-time index
    int ks_a = 0;             // K-step (within the tile) of the next fragments issued
    k64_u32x4 ar[3][2][MBW];  // [ring slot][chunk of the K-step][mb]
    auto issue_a = [&](auto slot_c) {
        constexpr int SL = decltype(slot_c)::value;
        if constexpr ((HIPANN_K64_ABLATE & 2) != 0) return;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t kc = 2 * ks_a + h;
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) ar[SL][h][mb] = Qw[kc * (K64_QM * 4) + qrow[mb]];
        }
        ks_a = ks_a + 1 < ns ? ks_a + 1 : 0;
    };
    auto issue_b = [&](int64_t g, int stage) {
        if constexpr ((HIPANN_K64_ABLATE & 1) != 0) return;
        k64_u32x4 *dst = smem_k64 + stage * K64_SU;
#pragma unroll
        for (int i = 0; i < PIECES; ++i) {
            const int inst = wave * PIECES + i;
            __builtin_amdgcn_global_load_lds((const void *)(Xb + g * K64_SU + inst * 64),
                                             (k64_lds_void *)(dst + inst * 64), 16, 0, 0);
        }
    };

    // the accumulators: int32 sums (I8) or fp32 (bf16), in their MFMA's own type
    using AccT = std::conditional_t<I8, k64_i32x4, k64_f32x4>;
    AccT acc[MBW][16];
#pragma unroll
    for (int mb = 0; mb < MBW; ++mb)
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) acc[mb][jb] = (AccT){0, 0, 0, 0};
    // ‖x‖² of tile tt, row 64·j + lane in xr[j] (0 for IP)
    float xr[4] = {0.f, 0.f, 0.f, 0.f};
    float xsc[4] = {1.f, 1.f, 1.f, 1.f};  // int8: the tile's row scales, row 64·j + lane in xsc[j]
    auto load_xn = [&](int64_t tt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t x = tt * K64_TN + 64 * j + lane;
            if constexpr (L2M) xr[j] = xnorm[x < N ? x : N - 1];  // rows past N: +inf at the use (G > 0: N > 0)
            if constexpr (I8) xsc[j] = xscale[x < N ? x : N - 1];
        }
    };
    constexpr int NXN = (L2M ? 4 : 0) + (I8 ? 4 : 0);  // load_xn's vector-memory ops
    // Per K-step g the vector-memory ops go out as A(g+2) (chunk 0) and B(g+3) (end of chunk 1); at its end A(g+1)
    // and B(g+1) must have landed, and B(g+2), A(g+2), B(g+3) — the three youngest groups — may stay in flight:
    // vmcnt(2·PIECES + 2·MBW).  Loads retire in issue order, so the query fragments must be issued before B(g+2)
    // for the wait not to cover it: with a one-K-step fragment lead (A(g+1) issued in K-step g, after B(g+2)) the
    // wait for A(g+1) also waited for B(g+2), and the tile pieces led by one K-step, not two.  The tile's ‖x‖² and
    // scales (NXN loads) go out at the start of K-step ns − 2 (its wait allows them in flight too; the epilogue's own
    // wait for them, two K-steps later, covers nothing younger than they are that is still needed).  The waits are the
    // builtin (s_waitcnt vmcnt(n) expcnt(7) lgkmcnt(15)), not inline asm: the compiler's wait pass must see them.
    constexpr int NA = (HIPANN_K64_ABLATE & 2) != 0 ? 0 : 2 * MBW;
    constexpr int NB_OPS = (HIPANN_K64_ABLATE & 1) != 0 ? 0 : PIECES;
    constexpr int kVm = 2 * NB_OPS + NA, kVmXn = kVm + NXN;
    static_assert(kVmXn < 64, "vmcnt field");
    constexpr unsigned kWaitStep = 0xF70u | (kVm & 15) | ((kVm >> 4) << 14);
    constexpr unsigned kWaitStepXn = 0xF70u | (kVmXn & 15) | ((kVmXn >> 4) << 14);

    auto clampg = [&](int64_t g) { return g < G ? g : G - 1; };  // past the end: the last K-step again, never read
    if (G > 0) {
        // the steady state's order: B(0), A(0), B(1), A(1), B(2)
        issue_b(0, 0);
        issue_a(std::integral_constant<int, 0>{});
        issue_b(clampg(1), 1);
        issue_a(std::integral_constant<int, 1>{});
        issue_b(clampg(2), 2);
    }
    __builtin_amdgcn_s_waitcnt(kWaitStep);  // B(0), A(0) landed (B(1), A(1), B(2) in flight)

    int ks = 0, stage = 0;
    int64_t t = t0;
    const int ks_xn = ns >= 2 ? ns - 2 : 0;  // the K-step (within a tile) that issues the tile's ‖x‖² / scales
    auto body = [&](int64_t g, auto slot_c) __attribute__((always_inline)) {
        constexpr int SL = decltype(slot_c)::value;
        const bool xn = ks == ks_xn;  // wave-uniform
        // K-step g landed (the wait at the end of the previous K-step), every wave done reading the stage about to
        // be refilled (g−2's): one barrier
        if constexpr ((HIPANN_K64_ABLATE & 8) == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // the tile's ‖x‖² (and int8 row scales) for the epilogue, once per tile (xnorm is deliberately not
        // __restrict__: a read-only noalias argument's loads get sunk into the epilogue's block, where the wait for
        // them is a vmcnt(0))
        if (xn) load_xn(t);
        __builtin_amdgcn_sched_barrier(0);
        const k64_u32x4 *Bb = smem_k64 + stage * K64_SU;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // A(g+2) spread over chunk 0's MFMAs, B(g+3) over chunk 1's last eight, after the K-step's last LDS
            // read (the compiler keeps LDS reads behind an LDS-DMA in program order).  Issued together after the
            // barrier instead, the eight vector-memory ops of all eight waves queue at once and hold back the
            // MFMAs (17.4 vs 16.6 ms with one K-step in flight).
            if (h == 0) issue_a(std::integral_constant<int, (SL + 2) % 3>{});
            // B fragment of rows 16·jb + m16, unit c = g4: slot c·256 + 16·jb + (m16 ^ 2c)
            const k64_u32x4 *Bc = Bb + h * K64_BU + g4 * K64_TN + (m16 ^ (g4 << 1));
            k64_b16x8 bf[16];
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) bf[jb] = __builtin_bit_cast(k64_b16x8, Bc[16 * jb]);
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) {
#pragma unroll
                for (int mb = 0; mb < MBW; ++mb) {
                    if constexpr (I8) {  // int32 sums carried in the accumulators' registers, bit for bit
                        const k64_i32x4 ai = __builtin_bit_cast(k64_i32x4, ar[SL][h][mb]);
                        const k64_i32x4 bi = __builtin_bit_cast(k64_i32x4, bf[jb]);
                        acc[mb][jb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai, bi, acc[mb][jb], 0, 0, 0);
                    } else {
                        acc[mb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(k64_b16x8, ar[SL][h][mb]),
                                                                              bf[jb], acc[mb][jb], 0, 0, 0);
                    }
                }
            }
            if (h == 1) issue_b(clampg(g + 3), stage < 2 ? stage + 3 : stage - 2);
            // schedule (same region): four LDS reads ahead, then one read per MBW MFMAs; the vector-memory ops (A
            // in chunk 0, B at the end of chunk 1) spread over the MFMAs
            const int NV = h == 0 ? 2 * MBW : PIECES;  // vector-memory ops of this chunk (constant once unrolled)
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int p = 0; p < 16; ++p) {
                __builtin_amdgcn_sched_group_barrier(0x008, MBW, 0);
                if (p < 12) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (h == 0) {
                    if (p % (16 / NV) == 1 % (16 / NV)) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
                } else if (p >= 16 - NV) {
                    __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
                }
            }
            // chunk fence: A(g+2) stays in chunk 0, B(g+3) at the end of chunk 1 (their order is what the counted
            // wait assumes)
            __builtin_amdgcn_sched_barrier(0);
        }
        // A(g+1), B(g+1) landed; B(g+2), A(g+2), B(g+3) (and this K-step's ‖x‖² / scales) stay in flight
        if (xn) __builtin_amdgcn_s_waitcnt(kWaitStepXn);
        else __builtin_amdgcn_s_waitcnt(kWaitStep);
        stage = stage + 1 < NB ? stage + 1 : 0;
    };
    // row blocks converted per epilogue part: 8 (32 values + 16 row terms beside the accumulators); STAG: 4, which frees
    // the 16 registers the staggered halves' longer fragment lifetimes need
#ifndef HIPANN_K64_EJ
#define HIPANN_K64_EJ 0
#endif
    constexpr int EJ = HIPANN_K64_EJ ? HIPANN_K64_EJ : (STAG ? 4 : 8);
    // the tile's epilogue (after its last K-step)
    auto epilogue = [&]() __attribute__((always_inline)) {
        const int64_t x0 = t * K64_TN;
        // s = 2·q·x − ‖x‖² (the filter's left side; the key follows from it with one more rounding, inside the
        // rerank bound's (d + 8)·2⁻²⁴ term); xr: row 64·j + l in lane l's xr[j].  Eight row blocks at a time (two
        // halves), each 16-query row block's accumulators converted, filtered and reset before the next: 32 values
        // and 16 row terms live besides the accumulators.
#pragma unroll
        for (int hf = 0; hf < 16 / EJ; ++hf) {
            float xvj[EJ], sxj[EJ];
#pragma unroll
            for (int j = 0; j < EJ; ++j) {
                const int jb = EJ * hf + j;
                const float xs = __shfl(xr[jb >> 2], 16 * (jb & 3) + m16);
                xvj[j] = x0 + 16 * jb + m16 < N ? xs : __builtin_inff();
                sxj[j] = I8 ? __shfl(xsc[jb >> 2], 16 * (jb & 3) + m16) : 1.f;
            }
            auto tile_mb = [&](auto mb_c) __attribute__((always_inline)) {
                constexpr int MB = decltype(mb_c)::value;
                if constexpr ((HIPANN_K64_ABLATE & 128) != 0 && !KEYS) {  // (tuning: the epilogue's cost — the
                    // accumulators consumed by one xor each and reset, no conversion or filter)
                    k64_f32x4 x = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < EJ; ++j) {
                        x = __builtin_elementwise_max(x, __builtin_convertvector(acc[MB][EJ * hf + j], k64_f32x4));
                        acc[MB][EJ * hf + j] = (AccT){0, 0, 0, 0};
                    }
                    cntv += x[0] + x[1] + x[2] + x[3] == 1234.5f ? 1 : 0;
                    return;
                }
                k64_f32x4 sm[EJ];
#pragma unroll
                for (int j = 0; j < EJ; ++j) {
                    const int jb = EJ * hf + j;
                    if constexpr (I8) {
                        // whole-vector reinterpret + convert: per-element extracts of the bit-cast i32 MFMA result
                        // were miscompiled (only element 0 of each accumulator was read; the others came from stale
                        // registers — found by the form's parity tests, every query with index % 4 != 0 wrong).
                        // Scalar fp32 (packed v_pk_mul/fma pairs pushed the kernel past 256 registers: spills,
                        // 8.26 vs 7.71 ms at 10M)
                        const k64_f32x4 v = __builtin_convertvector(acc[MB][jb], k64_f32x4);
                        if constexpr ((HIPANN_K64_ABLATE & 32) != 0) {  // (tuning: one query scale per tile)
                            const float cj = csq[0][0] * sxj[j];
#pragma unroll
                            for (int i = 0; i < 4; ++i) sm[j][i] = fmaf(cj, v[i], -xvj[j]);
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i) sm[j][i] = fmaf(csq[MB][i] * sxj[j], v[i], -xvj[j]);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) sm[j][i] = fmaf(2.f, acc[MB][jb][i], -xvj[j]);
                    }
                    if constexpr ((HIPANN_K64_ABLATE & 64) == 0) acc[MB][jb] = (AccT){0, 0, 0, 0};  // (64: tuning)
                }
                if constexpr (KEYS) {
                    // every key (L2: ‖q‖² − s clamped at 0; IP: −s/2) into the dense key matrix
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int64_t q = q0w + 16 * MB + i;
#pragma unroll
                        for (int j = 0; j < EJ; ++j) {
                            const int64_t x = x0 + 16 * (EJ * hf + j) + m16;
                            float key;
                            if (L2M) {
                                key = cth[MB][i] - sm[j][i];
                                key = key < 0.f ? 0.f : key;
                            } else {
                                key = -0.5f * sm[j][i];
                            }
                            if (q < nq && x < N) cand_d[q * N + x] = key;
                        }
                    }
                } else if constexpr ((HIPANN_K64_ABLATE & 4) != 0) {
                    cntv += sm[0][0] > 1e30f ? 1 : 0;  // (keeps the conversion live)
                } else {
                    // the lane's largest s per accumulator row (the filter's one compare per row); NaN-dropping max
                    k64_f32x4 mx = sm[0];
#pragma unroll
                    for (int j = 1; j < EJ; ++j) mx = __builtin_elementwise_max(mx, sm[j]);
                    k64_epilogue_row<L2M, MB, 0, EJ>(sm, mx[0], cth[MB], qnl, cntv, x0, cand_d, cand_i, cbase, cq, cap, lane, EJ * hf);
                    k64_epilogue_row<L2M, MB, 1, EJ>(sm, mx[1], cth[MB], qnl, cntv, x0, cand_d, cand_i, cbase, cq, cap, lane, EJ * hf);
                    k64_epilogue_row<L2M, MB, 2, EJ>(sm, mx[2], cth[MB], qnl, cntv, x0, cand_d, cand_i, cbase, cq, cap, lane, EJ * hf);
                    k64_epilogue_row<L2M, MB, 3, EJ>(sm, mx[3], cth[MB], qnl, cntv, x0, cand_d, cand_i, cbase, cq, cap, lane, EJ * hf);
                }
            };
            [&]<int... M>(std::integer_sequence<int, M...>) {
                (tile_mb(std::integral_constant<int, M>{}), ...);
            }(std::make_integer_sequence<int, MBW>{});
        }
        ++t;
    };

    // ---- STAG: the staggered schedule (see the template comment) ----
    // Both halves run ONE instruction stream — the half only selects operands (a branch per half duplicated the
    // accumulator updates and the allocator spilled ~1000 registers): per barrier interval g a chunk x, an epilogue
    // site, a chunk y, an epilogue site.  Early half: x = chunk 0 of K-step g, y = chunk 1 of g, epilogue after y when
    // g ends a tile.  Late half: x = chunk 1 of g − 1, epilogue after x when g − 1 ended a tile, y = chunk 0 of g.
    // Both issue the query fragments two K-steps ahead (A(g + 2) spread over chunk y, into slot SLP — read by the late
    // half's chunk x before) and the tile piece B(g + 3) at the end of y: the waits are the unstaggered schedule's.
    auto chunk_rt = [&](int h, int stg, const k64_u32x4 (&a)[MBW], auto vm_c, int sli_dummy, int64_t gb, int stgb,
                        auto sli_c) __attribute__((always_inline)) {
        constexpr int VM = decltype(vm_c)::value, SLI = decltype(sli_c)::value;
        (void)sli_dummy;
        __builtin_amdgcn_sched_barrier(0);
        const k64_u32x4 *Bc = smem_k64 + stg * K64_SU + h * K64_BU + g4 * K64_TN + (m16 ^ (g4 << 1));
        if constexpr ((VM & 1) != 0) issue_a(std::integral_constant<int, SLI>{});
        k64_b16x8 bf[16];
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) bf[jb] = __builtin_bit_cast(k64_b16x8, Bc[16 * jb]);
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) {
#pragma unroll
            for (int mb = 0; mb < MBW; ++mb) {
                if constexpr (I8) {
                    const k64_i32x4 ai = __builtin_bit_cast(k64_i32x4, a[mb]);
                    const k64_i32x4 bi = __builtin_bit_cast(k64_i32x4, bf[jb]);
                    acc[mb][jb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai, bi, acc[mb][jb], 0, 0, 0);
                } else {
                    acc[mb][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(k64_b16x8, a[mb]), bf[jb],
                                                                          acc[mb][jb], 0, 0, 0);
                }
            }
        }
        if constexpr ((VM & 2) != 0) issue_b(gb, stgb);
        constexpr int NAv = (VM & 1) != 0 ? 2 * MBW : 0, NBv = (VM & 2) != 0 ? PIECES : 0;
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            __builtin_amdgcn_sched_group_barrier(0x008, MBW, 0);
            if (p < 12) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if constexpr (NAv > 0) {
                if (p % (16 / NAv) == 1 % (16 / NAv)) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            }
            if constexpr (NBv > 0) {
                if (p >= 16 - NBv) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
#ifndef HIPANN_STAG_DBG
#define HIPANN_STAG_DBG 0
#endif
    const bool late = STAG && HIPANN_STAG_DBG != 2 && wave >= K64Geom<MBW>::W / 2;  // wave-uniform
    auto body_stag = [&](int64_t g, auto slot_c) __attribute__((always_inline)) {
        constexpr int SL = decltype(slot_c)::value;
        constexpr int SLP = (SL + 2) % 3, SLN = (SL + 1) % 3;  // slots of K-steps g − 1 and g + 1
        const bool xn = g < G && ks == ks_xn;
        if constexpr ((HIPANN_K64_ABLATE & 8) == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (xn) load_xn(t);
        __builtin_amdgcn_sched_barrier(0);
        const int stgb = stage < 2 ? stage + 3 : stage - 2;
        const int stprev = stage == 0 ? NB - 1 : stage - 1;
        k64_u32x4 ax[MBW], ay[MBW];
#pragma unroll
        for (int mb = 0; mb < MBW; ++mb) {
            ax[mb] = late ? ar[SLP][1][mb] : ar[SL][0][mb];
            ay[mb] = late ? ar[SL][0][mb] : ar[SL][1][mb];
        }
        if (late ? g >= 1 : g < G)
            chunk_rt(late ? 1 : 0, late ? stprev : stage, ax, std::integral_constant<int, 0>{}, 0, 0, 0,
                     std::integral_constant<int, SLN>{});
#if HIPANN_STAG_DBG != 1
        if (late && g >= 1 && ks == 0) {  // g − 1 ended a tile (g = G included: G is whole tiles)
            // the epilogue's VALU at a lower priority than the partner's MFMA issue (MI355X_MICROARCH.md, two waves per
            // SIMD, item 2: arbitration by priority, then age)
            __builtin_amdgcn_s_setprio(0);
            epilogue();
            __builtin_amdgcn_s_setprio(2);
        }
#endif
        if (g < G)
            chunk_rt(late ? 0 : 1, stage, ay, std::integral_constant<int, 3>{}, 0, clampg(g + 3), stgb,
                     std::integral_constant<int, SLP>{});
        if (!late && g < G && ks == ns - 1) {
            __builtin_amdgcn_s_setprio(0);
            epilogue();
            __builtin_amdgcn_s_setprio(2);
        }
        // A(g + 1), B(g + 1) landed; B(g + 2), A(g + 2), B(g + 3) (and the norms issued at the top) may stay in flight
        if (xn) __builtin_amdgcn_s_waitcnt(kWaitStepXn);
        else __builtin_amdgcn_s_waitcnt(kWaitStep);
        ks = ks + 1 < ns ? ks + 1 : 0;
        stage = stage + 1 < NB ? stage + 1 : 0;
    };
    if constexpr (STAG) {
        __builtin_amdgcn_s_setprio(2);
        for (int64_t g = 0; g <= G; g += 3) {
            body_stag(g, std::integral_constant<int, 0>{});
            if (g + 1 <= G) body_stag(g + 1, std::integral_constant<int, 1>{});
            if (g + 2 <= G) body_stag(g + 2, std::integral_constant<int, 2>{});
        }
    } else {
        auto step = [&](int64_t g, auto slot_c) __attribute__((always_inline)) {
            body(g, slot_c);
            if (++ks == ns) {
                ks = 0;
                epilogue();
            }
        };
        for (int64_t g = 0; g < G; g += 3) {
            step(g, std::integral_constant<int, 0>{});
            if (g + 1 < G) step(g + 1, std::integral_constant<int, 1>{});
            if (g + 2 < G) step(g + 2, std::integral_constant<int, 2>{});
        }
    }
    // no LDS-DMA copy may land after the block's LDS is handed to the next block
    __builtin_amdgcn_s_waitcnt(0xF70u);
    if (!KEYS && lane < QW && qlane < nq) cand_n[qlane * nsplit + split] = cntv;
}

// Candidates of query q, one split per lane: round j offers entry j of splits s0 + lane (64 splits at a time),
// the round's loads issued together ahead of its offers (a query holds ≈10-30 per split: ≈max-count rounds).
template <bool WITH_IDS, typename F>
__device__ __forceinline__ bool cand_offer_all(const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                                               const int *__restrict__ cand_n, int nsplit, int cap, int64_t q,
                                               int lane, F offer) {
    bool over = false;
    for (int s0 = 0; s0 < nsplit; s0 += 64) {
        const int s = s0 + lane;
        const int nr = s < nsplit ? cand_n[q * nsplit + s] : 0;
        over |= nr > cap;
        const int n = nr < cap ? nr : cap;
        int mx = n;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        const int64_t base = (q * nsplit + s) * (int64_t)cap;
        constexpr int U = 8;  // entries per lane loaded ahead of their offers
        for (int j0 = 0; j0 < mx; j0 += U) {
            float v[U];
            int id[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool ok = j0 + u < n;
                v[u] = ok ? cand_d[base + j0 + u] : __builtin_inff();
                id[u] = WITH_IDS && ok ? cand_i[base + j0 + u] : 0x7fffffff;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (j0 + u < mx) offer(v[u], WITH_IDS ? id[u] : lane);
        }
    }
    return __ballot(over) != 0ull;
}

// The k-th smallest candidate key of each query over all splits (its bound for the next pass), with the
// margin of flat_bf16_seed, never above the current bound.  One wave per query.
__global__ void __launch_bounds__(256) flat_cand_bound(const float *__restrict__ cand_d, const int *__restrict__ cand_n,
                                                       int nsplit, int cap, int64_t nq, int k,
                                                       float *__restrict__ bound) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<1, int> L;
    L.init();
    cand_offer_all<false>(cand_d, nullptr, cand_n, nsplit, cap, q, lane,
                          [&](float v, int id) { L.offer(v, id, k - 1); });
    if (lane == 0) {
        const float t = readlane_f(L.d[0], k - 1);
        const float tm = t == __builtin_inff() ? t : fmaxf(t * (1.f + 0x1p-20f), t + 0x1p-100f);
        bound[q] = fminf(bound[q], tm);
    }
}

// Each query's k best candidates (key, row) over all splits, ascending, into out_[di][q·k + j] — the list the
// rerank merges (nsplit = 1).  A query whose buffer overflowed in some split is appended to flagged (the exact
// fallback re-runs it).  One wave per query.
__global__ void __launch_bounds__(256) flat_cand_select(const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                                                        const int *__restrict__ cand_n, int nsplit, int cap, int64_t nq,
                                                        int k, float *__restrict__ out_d, int *__restrict__ out_i,
                                                        int *__restrict__ nflag, int *__restrict__ flagged) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<1, int> L;
    L.init();
    const bool over = cand_offer_all<true>(cand_d, cand_i, cand_n, nsplit, cap, q, lane,
                                           [&](float v, int id) { L.offer(v, id, k - 1); });
    // an overflowed query gets an all-pad list: the rerank then finds no candidate and does not flag it a second
    // time (flagged holds nq entries)
    if (lane < k) {
        out_d[q * k + lane] = over ? __builtin_inff() : L.d[0];
        out_i[q * k + lane] = over ? 0x7fffffff : L.id[0];
    }
    if (over && lane == 0) flagged[atomicAdd(nflag, 1)] = (int)q;
}

// ---- the candidate kernels narrowed (one 256-thread block per query) ---------------------------------------
// flat_cand_bound / flat_cand_select offer every buffered candidate to a wave list (≈ 26 per (query, split)
// cell at 10M rows, 64 splits: 26 dependent insert rounds of one wave per query — 26 + 72 µs per 1024-query
// C2 batch).  Here the block's 4 waves each take every 4th entry of the query's cells (lane = split), and the
// order statistic is narrowed as in flat_keys_kth: T_hi = the k-th smallest per-thread minimum, the entries
// ≤ T_hi (key bits + cell slot) go to an LDS list, and wave 0 finishes on ≤ KTH_CAP entries.  A longer list (or
// k > 64) falls back to the wave list in wave 0.  Same bound bit for bit; the same k (key, row) pairs in the same
// order (ties by row, as the wave list).
constexpr int CN_CAP = 256;
struct CandNarrow {
    unsigned key[CN_CAP];
    int slot[CN_CAP];
    int n;
    int part[4];
    int over;
};
__device__ __forceinline__ unsigned cn_bits(float v) {
    const float f = v == 0.f ? 0.f : v;
    const unsigned b = __float_as_uint(f);
    return v == v ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
}
__device__ __forceinline__ float cn_unbits(unsigned b) {
    return __uint_as_float((b & 0x80000000u) ? (b & 0x7fffffffu) : ~b);
}
// block-wide: smallest t with #{m_thread ≤ t} ≥ k over the block's 256 values (32 rounds, one ballot per wave)
__device__ __forceinline__ unsigned cn_block_kth(unsigned m, int k, int *part) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned lo = 0u, hi = 0xffffffffu;
    while (lo < hi) {
        const unsigned mid = lo + (hi - lo) / 2u;
        const int c = (int)__popcll(__ballot(m <= mid));
        __syncthreads();
        if (lane == 0) part[wv] = c;
        __syncthreads();
        if (part[0] + part[1] + part[2] + part[3] >= k) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}
// the query's entries ≤ T_hi into S (S.n may exceed CN_CAP: then only the count is exact); S.over = some cell
// overflowed its capacity
__device__ __forceinline__ void cand_narrow(const float *__restrict__ cand_d, const int *__restrict__ cand_n,
                                            int nsplit, int cap, int64_t q, int k, CandNarrow &S) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) { S.n = 0; S.over = 0; }
    unsigned m = 0xffffffffu;
    bool over = false;
    for (int s0 = 0; s0 < nsplit; s0 += 64) {
        const int s = s0 + lane;
        const int nr = s < nsplit ? cand_n[q * nsplit + s] : 0;
        over |= nr > cap;
        const int n = nr < cap ? nr : cap;
        const int64_t base = (q * nsplit + s) * (int64_t)cap;
#pragma unroll 4
        for (int j = wv; j < n; j += 4) m = min(m, cn_bits(cand_d[base + j]));
    }
    const unsigned th = cn_block_kth(m, k, S.part);  // its barriers order the S.n / S.over reset
    if (__ballot(over) != 0ull && lane == 0) S.over = 1;
    for (int s0 = 0; s0 < nsplit; s0 += 64) {
        const int s = s0 + lane;
        const int nr = s < nsplit ? cand_n[q * nsplit + s] : 0;
        const int n = nr < cap ? nr : cap;
        const int64_t base = (q * nsplit + s) * (int64_t)cap;
        for (int j = wv; j < n; j += 4) {
            const unsigned b = cn_bits(cand_d[base + j]);
            if (b <= th) {
                const int p = atomicAdd(&S.n, 1);
                if (p < CN_CAP) { S.key[p] = b; S.slot[p] = s * cap + j; }
            }
        }
    }
    __syncthreads();
}
// wave 0: the k-th smallest key bits of the S list (n ≤ CN_CAP entries); ~0u when n < k
__device__ __forceinline__ unsigned cn_wave_kth(const CandNarrow &S, int n, int k, unsigned (&v)[CN_CAP / 64]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < CN_CAP / 64; ++i) v[i] = lane + 64 * i < n ? S.key[lane + 64 * i] : 0xffffffffu;
    if (n < k) return 0xffffffffu;
    unsigned lo = 0u, hi = 0xffffffffu;
    while (lo < hi) {
        const unsigned mid = lo + (hi - lo) / 2u;
        int c = 0;
#pragma unroll
        for (int i = 0; i < CN_CAP / 64; ++i) c += (int)__popcll(__ballot(v[i] <= mid));
        if (c >= k) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}

__global__ void __launch_bounds__(256) flat_cand_bound_nw(const float *__restrict__ cand_d, const int *__restrict__ cand_n,
                                                          int nsplit, int cap, int64_t nq, int k,
                                                          float *__restrict__ bound) {
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    __shared__ CandNarrow S;
    cand_narrow(cand_d, cand_n, nsplit, cap, q, k, S);
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const int n = S.n;
    float t;
    if (n <= CN_CAP) {
        unsigned v[CN_CAP / 64];
        const unsigned b = cn_wave_kth(S, n, k, v);
        t = b == 0xffffffffu ? __builtin_inff() : cn_unbits(b);
    } else {  // a long tie run at T_hi: the wave list over every entry
        WaveList<1, int> L;
        L.init();
        cand_offer_all<false>(cand_d, nullptr, cand_n, nsplit, cap, q, lane,
                              [&](float v, int id) { L.offer(v, id, k - 1); });
        t = readlane_f(L.d[0], k - 1);
    }
    if (lane == 0) {
        const float tm = t == __builtin_inff() ? t : fmaxf(t * (1.f + 0x1p-20f), t + 0x1p-100f);
        bound[q] = fminf(bound[q], tm);
    }
}

__global__ void __launch_bounds__(256) flat_cand_select_nw(const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                                                           const int *__restrict__ cand_n, int nsplit, int cap,
                                                           int64_t nq, int k, float *__restrict__ out_d,
                                                           int *__restrict__ out_i, int *__restrict__ nflag,
                                                           int *__restrict__ flagged) {
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    __shared__ CandNarrow S;
    __shared__ unsigned sel_k[64];
    __shared__ int sel_r[64];
    cand_narrow(cand_d, cand_n, nsplit, cap, q, k, S);
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const int n = S.n;
    const int64_t cbase = q * nsplit * (int64_t)cap;
    float kk = __builtin_inff();
    int row = 0x7fffffff;
    int nsel = 0;
    if (S.over) {  // as flat_cand_select: an all-pad list, the query flagged for the exact fallback
        if (lane == 0) flagged[atomicAdd(nflag, 1)] = (int)q;
    } else if (n <= 64) {
        if (lane < n) {
            kk = cn_unbits(S.key[lane]);
            row = cand_i[cbase + S.slot[lane]];
        }
        wave_rank_sort(kk, row, n);
        nsel = n < k ? n : k;
    } else if (n <= CN_CAP && k <= 64) {
        // T = the k-th key; all keys < T, then the keys == T with the smallest rows up to k (ties by row)
        unsigned v[CN_CAP / 64];
        const unsigned T = cn_wave_kth(S, n, k, v);
        int r[CN_CAP / 64];
        int clt = 0;
#pragma unroll
        for (int i = 0; i < CN_CAP / 64; ++i) {
            r[i] = v[i] == T && lane + 64 * i < n ? cand_i[cbase + S.slot[lane + 64 * i]] : 0x7fffffff;
            clt += (int)__popcll(__ballot(v[i] < T));
        }
        const int need = k - clt;  // ≥ 1 tied entries to take
        unsigned lo = 0u, hi = 0x7fffffffu;  // the need-th smallest row among the ties (rows are distinct)
        while (lo < hi) {
            const unsigned mid = lo + (hi - lo) / 2u;
            int c = 0;
#pragma unroll
            for (int i = 0; i < CN_CAP / 64; ++i) c += (int)__popcll(__ballot((unsigned)r[i] <= mid));
            if (c >= need) hi = mid;
            else lo = mid + 1u;
        }
        const unsigned long long lt = (1ull << lane) - 1ull;
        int base = 0;
#pragma unroll
        for (int i = 0; i < CN_CAP / 64; ++i) {
            const bool take = lane + 64 * i < n && (v[i] < T || (v[i] == T && (unsigned)r[i] <= lo));
            const unsigned long long mk = __ballot(take);
            if (take) {
                const int p = base + (int)__popcll(mk & lt);
                sel_k[p] = v[i];
                sel_r[p] = lane + 64 * i;
            }
            base += (int)__popcll(mk);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < k) {
            kk = cn_unbits(sel_k[lane]);
            row = cand_i[cbase + S.slot[sel_r[lane]]];
        }
        wave_rank_sort(kk, row, k);
        nsel = k;
    } else {  // a long tie run at T_hi: the wave list over every entry
        WaveList<1, int> L;
        L.init();
        cand_offer_all<true>(cand_d, cand_i, cand_n, nsplit, cap, q, lane,
                             [&](float v, int id) { L.offer(v, id, k - 1); });
        kk = L.d[0];
        row = L.id[0];
        nsel = k;
    }
    if (lane < k) {
        out_d[q * k + lane] = lane < nsel ? kk : __builtin_inff();
        out_i[q * k + lane] = lane < nsel ? row : 0x7fffffff;
    }
}

// The k-th smallest of each query's S sample keys (keys[q·S + j]), with the margin of flat_bf16_seed: the seed
// bound of the bounded passes.  One 256-thread block per query, the keys in registers (S ≤ 256·KPT).  A bisection
// on order-preserving bits over all 256·KPT registers costs 32 × KPT compares per thread (50 µs per 1024-query
// batch at 16K keys: VALU-bound), so the order statistic is narrowed first: T_hi = the k-th smallest of the 256
// per-thread minima (k of the keys lie at or below it, so the answer is ≤ T_hi; for i.i.d. keys ≈ 34 keys of 16K
// lie below it at k = 32, ≈ 74 at k = 64), the keys ≤ T_hi go to an LDS list, and one wave bisects that list.  A list longer than
// KTH_CAP falls back to the full bisection on [0, T_hi].  Same result as the full bisection, bit for bit.
constexpr int KTH_KPT = 64;
constexpr int KTH_CAP = 256;  // the one-wave finish: 4 list entries per lane
template <int KPT>
__global__ void __launch_bounds__(256) flat_keys_kth(const float *__restrict__ keys, int S, int64_t nq, int k,
                                                     float *__restrict__ bound, int narrow) {
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    __shared__ int part[4];
    __shared__ unsigned cand[KTH_CAP];
    __shared__ int ncand;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned u[KPT];
    unsigned m = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const int c = j * 256 + (int)threadIdx.x;
        const unsigned b = c < S ? __float_as_uint(keys[q * S + c]) : 0x7f800000u;  // +inf past S
        u[j] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);                        // order-preserving
        m = min(m, u[j]);
    }
    if (threadIdx.x == 0) ncand = 0;
    unsigned lo = 0u, hi = 0xffffffffu;  // smallest t with #{u ≤ t} ≥ k
    auto finish = [&]() {
        if (threadIdx.x == 0) {
            const unsigned b = (lo & 0x80000000u) ? (lo & 0x7fffffffu) : ~lo;
            const float t = __uint_as_float(b);
            bound[q] = t == __builtin_inff() ? t : fmaxf(t * (1.f + 0x1p-20f), t + 0x1p-100f);
        }
    };
    if (narrow && k <= 256) {
        // T_hi: the k-th smallest thread minimum (one ballot per wave per round)
        while (lo < hi) {
            const unsigned mid = lo + (hi - lo) / 2u;
            const int c = (int)__popcll(__ballot(m <= mid));
            __syncthreads();
            if (lane == 0) part[wv] = c;
            __syncthreads();
            const int tot = part[0] + part[1] + part[2] + part[3];
            if (tot >= k) hi = mid;
            else lo = mid + 1u;
        }
        const unsigned th = lo;
#pragma unroll
        for (int j = 0; j < KPT; ++j)
            if (u[j] <= th) {
                const int p = atomicAdd(&ncand, 1);
                if (p < KTH_CAP) cand[p] = u[j];
            }
        __syncthreads();
        const int nc = ncand;
        if (nc <= KTH_CAP) {
            if (wv != 0) return;
            unsigned v[KTH_CAP / 64];
#pragma unroll
            for (int i = 0; i < KTH_CAP / 64; ++i) v[i] = lane + 64 * i < nc ? cand[lane + 64 * i] : 0xffffffffu;
            lo = 0u;
            hi = th;  // mid < hi ≤ th never counts the ~0 pads
            while (lo < hi) {
                const unsigned mid = lo + (hi - lo) / 2u;
                int c = 0;
#pragma unroll
                for (int i = 0; i < KTH_CAP / 64; ++i) c += (int)__popcll(__ballot(v[i] <= mid));
                if (c >= k) hi = mid;
                else lo = mid + 1u;
            }
            finish();
            return;
        }
        lo = 0u;
        hi = th;
    }
    while (lo < hi) {
        const unsigned mid = lo + (hi - lo) / 2u;
        int c = 0;
#pragma unroll
        for (int j = 0; j < KPT; ++j) c += u[j] <= mid ? 1 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        __syncthreads();
        if (lane == 0) part[wv] = c;
        __syncthreads();
        const int tot = part[0] + part[1] + part[2] + part[3];
        if (tot >= k) hi = mid;
        else lo = mid + 1u;
    }
    finish();
}

int flat_keys_kth_max() { return 256 * KTH_KPT; }

void launch_flat_keys_kth(const float *keys, int S, int64_t nq, int k, float *bound, hipStream_t st) {
    if (nq <= 0) return;
    HIPANN_REQUIRE(S >= k && S <= 256 * KTH_KPT, "flat_keys_kth: sample size");
    // HIPANN_FLAT_KTH_NARROW=0 (A/B): the full 32-round bisection over every register
    static const int narrow = [] { const char *e = std::getenv("HIPANN_FLAT_KTH_NARROW"); return e ? std::atoi(e) : 1; }();
    // keys per thread sized to the sample
    if (S <= 256 * 16)
        hipLaunchKernelGGL(flat_keys_kth<16>, dim3((unsigned)nq), dim3(256), 0, st, keys, S, nq, k, bound, narrow);
    else
        hipLaunchKernelGGL(flat_keys_kth<KTH_KPT>, dim3((unsigned)nq), dim3(256), 0, st, keys, S, nq, k, bound, narrow);
    HIPANN_CHECK(hipGetLastError());
}

// test hook (tests/test_flat_kth_gpu.py): the seed k-th pass on device keys, narrowed (narrow = 1) or the full
// bisection (0); synchronous; 0 on success, -1 on a bad shape or a HIP error
extern "C" int hipann_debug_flat_keys_kth(const float *keys, int S, int64_t nq, int k, float *bound, int narrow) {
    if (nq <= 0 || k <= 0 || S < k || S > 256 * KTH_KPT || !keys || !bound) return -1;
    if (S <= 256 * 16)
        hipLaunchKernelGGL(flat_keys_kth<16>, dim3((unsigned)nq), dim3(256), 0, 0, keys, S, nq, k, bound, narrow);
    else
        hipLaunchKernelGGL(flat_keys_kth<KTH_KPT>, dim3((unsigned)nq), dim3(256), 0, 0, keys, S, nq, k, bound, narrow);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

bool flat_bf16_k64_supported(int nk, int k) { return nk % 2 == 0 && k <= 64; }

// ---- int8 image (form kFlatI8Exact) ------------------------------------------------------------------
// Per row: s = max|x| / 127 and x̂ = clamp(rint(x / s), ±127) (s = 0: a zero row); the tiled image has the bf16
// image's geometry with 64 dims per 64-B chunk row (16-B unit c of chunk kc = dims 64·kc + 16c .. +15), the chunk
// count rounded up to even (the K-step is two chunks) and zero-filled.
constexpr int I8_KC = 64;
int flat_i8_nk(int d) {
    const int nk = (d + I8_KC - 1) / I8_KC;
    return nk + (nk & 1);
}
size_t flat_i8_img_bytes(int64_t n, int d, int R) {
    return (size_t)ceil_div(std::max<int64_t>(n, 1), R) * flat_i8_nk(d) * R * 4 * 16;
}
__device__ __forceinline__ int i8_quant(float x, float s) {
    return s > 0.f ? (int)fminf(fmaxf(rintf(x / s), -127.f), 127.f) : 0;
}

// one wave per row: scale[row] = max|x| / 127, resid[row] = ‖x − s·x̂‖ (×1.0001: the fp32 sum of d exact-ish squares)
__global__ void __launch_bounds__(256) i8_row_scale(const float *__restrict__ X, int64_t n, int d,
                                                    float *__restrict__ scale, float *__restrict__ resid) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    const float *x = X + row * (int64_t)d;
    float m = 0.f;
    for (int e = lane; e < d; e += 64) m = fmaxf(m, fabsf(x[e]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float s = m > 0.f && m < 3.0e38f ? m / 127.f : 0.f;
    float r2 = 0.f;
    for (int e = lane; e < d; e += 64) {
        const float r = x[e] - s * (float)i8_quant(x[e], s);
        r2 = fmaf(r, r, r2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r2 += __shfl_xor(r2, o);
    if (lane == 0) {
        scale[row] = s;
        resid[row] = m < 3.0e38f ? sqrtf(r2) * 1.0001f : __builtin_inff();  // non-finite rows: no bound
    }
}

// unit u = ((t·nk + kc)·4 + c)·R + (row ^ 2c), one thread per unit (16 int8 values)
__global__ void __launch_bounds__(256) i8_tile_rows(const float *__restrict__ X, const float *__restrict__ scale,
                                                    int64_t n, int d, int R, int nk, int64_t total,
                                                    uint4 *__restrict__ out) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= total) return;
    const int rr = (int)(u % R);
    int64_t rest = u / R;
    const int c = (int)(rest & 3);
    rest >>= 2;
    const int kc = (int)(rest % nk);
    const int64_t t = rest / nk;
    const int row = rr ^ (c << 1);
    const int64_t grow = t * R + row;
    const int dim0 = kc * I8_KC + 16 * c;
    unsigned w[4] = {0u, 0u, 0u, 0u};
    if (grow < n) {
        const float s = scale[grow];
        const float *x = X + grow * (int64_t)d;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int v = dim0 + i < d ? i8_quant(x[dim0 + i], s) : 0;
            w[i >> 2] |= ((unsigned)v & 0xffu) << (8 * (i & 3));
        }
    }
    out[u] = make_uint4(w[0], w[1], w[2], w[3]);
}

// The batch's int8 query preparation in one launch (the bounded passes' queries): one wave per row of the padded
// tiles — ‖q‖² (optional, row_norms_f32's order and bits), i8_row_scale's scale and residual (same order), and the
// row's units of i8_tile_rows' image (padding rows: zero units).  Three dependent launches were ≈ 16 µs of kernels
// plus their host launch time at the start of every C2 search (r05 runtime trace).
__global__ void __launch_bounds__(256) i8_query_prep(const float *__restrict__ X, int64_t n, int d, int vec4,
                                                     float *__restrict__ qn, float *__restrict__ scale,
                                                     float *__restrict__ resid, int R, int nk, int64_t npad,
                                                     uint4 *__restrict__ out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= npad) return;
    const int lane = threadIdx.x & 63;
    const int64_t t = row / R;
    const int rin = (int)(row - t * R);
    if (row >= n) {  // a padding row of the last tile
        for (int uc = lane; uc < nk * 4; uc += 64) {
            const int kc = uc >> 2, c = uc & 3;
            out[((t * nk + kc) * 4 + c) * R + (rin ^ (c << 1))] = make_uint4(0u, 0u, 0u, 0u);
        }
        return;
    }
    const float *x = X + row * (int64_t)d;
    if (qn) {
        float s2 = 0.f;
        if (vec4) {
            const float4 *p4 = reinterpret_cast<const float4 *>(x);
            for (int j = lane; j < (d >> 2); j += 64) {
                const float4 v = p4[j];
                s2 = fmaf(v.x, v.x, s2); s2 = fmaf(v.y, v.y, s2); s2 = fmaf(v.z, v.z, s2); s2 = fmaf(v.w, v.w, s2);
            }
        } else {
            for (int j = lane; j < d; j += 64) s2 = fmaf(x[j], x[j], s2);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
        if (lane == 0) qn[row] = s2;
    }
    float m = 0.f;
    for (int e = lane; e < d; e += 64) m = fmaxf(m, fabsf(x[e]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float s = m > 0.f && m < 3.0e38f ? m / 127.f : 0.f;
    float r2 = 0.f;
    for (int e = lane; e < d; e += 64) {
        const float r = x[e] - s * (float)i8_quant(x[e], s);
        r2 = fmaf(r, r, r2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r2 += __shfl_xor(r2, o);
    if (lane == 0) {
        scale[row] = s;
        resid[row] = m < 3.0e38f ? sqrtf(r2) * 1.0001f : __builtin_inff();
    }
    for (int uc = lane; uc < nk * 4; uc += 64) {
        const int kc = uc >> 2, c = uc & 3;
        const int dim0 = kc * I8_KC + 16 * c;
        unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int v = dim0 + i < d ? i8_quant(x[dim0 + i], s) : 0;
            w[i >> 2] |= ((unsigned)v & 0xffu) << (8 * (i & 3));
        }
        out[((t * nk + kc) * 4 + c) * R + (rin ^ (c << 1))] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

void launch_i8_query_prep(const float *X, int64_t n, int d, float *qn, float *scale, float *resid, int R, void *out,
                          hipStream_t st) {
    if (n <= 0) return;
    const int nk = flat_i8_nk(d);
    const int64_t npad = ceil_div(n, R) * R;
    const int vec4 = (d % 4 == 0) && ((uintptr_t)X % 16 == 0);
    hipLaunchKernelGGL(i8_query_prep, dim3((unsigned)ceil_div(npad, 4)), dim3(256), 0, st, X, n, d, vec4, qn, scale,
                       resid, R, nk, npad, static_cast<uint4 *>(out));
    HIPANN_CHECK(hipGetLastError());
}

void launch_i8_row_scale(const float *X, int64_t n, int d, float *scale, float *resid, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(i8_row_scale, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, X, n, d, scale, resid);
    HIPANN_CHECK(hipGetLastError());
}

void launch_i8_tile_rows(const float *X, const float *scale, int64_t n, int d, int R, void *out, hipStream_t st) {
    const int nk = flat_i8_nk(d);
    const int64_t total = ceil_div(std::max<int64_t>(n, 1), R) * nk * R * 4;
    hipLaunchKernelGGL(i8_tile_rows, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st, X, scale, n, d, R, nk,
                       total, static_cast<uint4 *>(out));
    HIPANN_CHECK(hipGetLastError());
}


// ---- small batches (nq < 20, FAISS's direct-form path) over the int8 image ---------------------------------
// flat_i8_scan: the extension's per-query call (faiss_index.cpp:737, search(1, …)) streams the int8 image instead
// of the fp32 rows — a quarter of the bytes.  Lane = database row: a wave takes 64-row groups (a quarter of a
// 256-row tile: each 16-B unit of the group is one coalesced 1-KiB read, the rows' XOR swizzle permutes lanes
// within it), accumulates the exact int32 dot products with the queries' int8 images (v_dot4, 4 per unit; the
// query units in LDS, read as broadcasts), and offers key = ‖q‖² + ‖x‖² − 2·s_q·s_x·dot (IP: −s_q·s_x·dot) to one
// 64-deep wave list per query.  The lists are a filter: flat_i8_group_merge + ivf_rerank_topk recompute the
// survivors in the direct fp32 form and certify them with the int8 residual bound of the batched form 5.
constexpr int I8S_K = 64;  // filter depth (the batched form 5's)
__device__ __forceinline__ int i8s_dot16(uint4 x, uint4 q, int acc) {
    acc = __builtin_amdgcn_sdot4((int)x.x, (int)q.x, acc, false);
    acc = __builtin_amdgcn_sdot4((int)x.y, (int)q.y, acc, false);
    acc = __builtin_amdgcn_sdot4((int)x.z, (int)q.z, acc, false);
    return __builtin_amdgcn_sdot4((int)x.w, (int)q.w, acc, false);
}
template <int NQ, bool IP>
__global__ void __launch_bounds__(256)
flat_i8_scan(const uint4 *__restrict__ qimg, const float *__restrict__ qscale, const float *__restrict__ qnorm,
             const uint4 *__restrict__ ximg, const float *__restrict__ xscale, const float *xnorm, int64_t N, int nk,
             int64_t groups_per_wave, float *__restrict__ part_d, int *__restrict__ part_i) {
    extern __shared__ uint4 i8s_q[];  // [NQ][nk][4] query units
    for (int i = threadIdx.x; i < NQ * nk * 4; i += 256) i8s_q[i] = qimg[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t ngroups = (N + 63) / 64;
    const int64_t g0 = gw * groups_per_wave;
    const int64_t g1 = g0 + groups_per_wave < ngroups ? g0 + groups_per_wave : ngroups;
    float qsc[NQ], qn[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
        qsc[qi] = qscale[qi];
        qn[qi] = IP ? 0.f : qnorm[qi];
    }
    WaveList<1, int> L[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) L[qi].init();
    for (int64_t g = g0; g < g1; ++g) {
        const int64_t t = g >> 2;
        const int rin = 64 * (int)(g & 3) + lane;  // row within the tile
        const int64_t row = t * 256 + rin;
        const bool valid = row < N;
        const uint4 *tb = ximg + t * (int64_t)nk * 4 * 256;
        int acc[NQ];
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) acc[qi] = 0;
        for (int kc = 0; kc < nk; kc += 2) {  // nk is even (flat_i8_nk)
            uint4 xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = u & 3;
                xv[u] = tb[((int64_t)(kc + (u >> 2)) * 4 + c) * 256 + (rin ^ (c << 1))];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) acc[qi] = i8s_dot16(xv[u], i8s_q[(qi * nk + kc) * 4 + u], acc[qi]);
        }
        const int64_t rr = valid ? row : N - 1;
        const float sx = xscale[rr], xv2 = IP ? 0.f : xnorm[rr];
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) {
            const float s = qsc[qi] * sx * (float)acc[qi];
            float key;
            if (IP) {
                key = -s;
            } else {
                key = fmaf(-2.f, s, qn[qi] + xv2);
                key = key < 0.f ? 0.f : key;
            }
            L[qi].offer(valid ? key : __builtin_inff(), valid ? (int)row : IdTraits<int>::pad(), I8S_K - 1);
        }
    }
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
        part_d[(gw * NQ + qi) * I8S_K + lane] = L[qi].d[0];
        part_i[(gw * NQ + qi) * I8S_K + lane] = L[qi].id[0];
    }
}

// The scan's per-wave lists [wave][q][64] merged in groups of `per` waves into [q][group][64] (the rerank's
// query-major slot lists).  One wave per (group, query); four lists' loads issued ahead of their offers.
__global__ void __launch_bounds__(256)
flat_i8_group_merge(const float *__restrict__ pd, const int *__restrict__ pi, int nw, int nq, int per, int ngroup,
                    float *__restrict__ od, int *__restrict__ oi) {
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= (int64_t)ngroup * nq) return;
    const int q = (int)(item / ngroup), grp = (int)(item - (int64_t)q * ngroup);
    const int lane = threadIdx.x & 63;
    WaveList<1, int> L;
    L.init();
    const int w0 = grp * per, w1 = w0 + per < nw ? w0 + per : nw;
    for (int w = w0; w < w1; w += 4) {
        float v[4];
        int id[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool ok = w + u < w1;
            const int64_t off = ((int64_t)(ok ? w + u : w0) * nq + q) * I8S_K + lane;
            v[u] = ok ? pd[off] : __builtin_inff();
            id[u] = ok ? pi[off] : IdTraits<int>::pad();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) L.offer(v[u], id[u], I8S_K - 1);
    }
    od[((int64_t)q * ngroup + grp) * I8S_K + lane] = L.d[0];
    oi[((int64_t)q * ngroup + grp) * I8S_K + lane] = L.id[0];
}

// The queries' int8 units, [q][kc][c] (16 dims each, zero past d), quantized with their scales (i8_row_scale).
__global__ void __launch_bounds__(256) i8_query_units(const float *__restrict__ Q, const float *__restrict__ scale,
                                                      int64_t nq, int d, int nk, uint4 *__restrict__ out) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= nq * nk * 4) return;
    const int64_t q = u / (nk * 4);
    const int rem = (int)(u - q * nk * 4), kc = rem >> 2, c = rem & 3;
    const float s = scale[q];
    const float *x = Q + q * (int64_t)d;
    const int dim0 = kc * I8_KC + 16 * c;
    unsigned w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int v = dim0 + i < d ? i8_quant(x[dim0 + i], s) : 0;
        w[i >> 2] |= ((unsigned)v & 0xffu) << (8 * (i & 3));
    }
    out[u] = make_uint4(w[0], w[1], w[2], w[3]);
}

int flat_i8_scan_k() { return I8S_K; }
// up to 16 queries the per-query lists stay in registers (17-19 spill to scratch: those batches take the fp32 scan)
int flat_i8_scan_max_nq() { return 16; }
int64_t flat_i8_scan_waves(int64_t n) {
    // ≈ 2048 waves (8 per CU), ≥ 16 groups of 64 rows each; a multiple of 4 — the grid is whole 4-wave blocks and
    // every wave writes its lists, so the caller's part buffers (nw·nq·64) must cover every launched wave (waves
    // past the last group write all-pad lists)
    const int64_t ngroups = (n + 63) / 64;
    return (std::max<int64_t>(1, std::min<int64_t>(2048, ngroups / 16)) + 3) / 4 * 4;
}
void launch_flat_i8_scan(const float *Q, int64_t nq, int d, int metric, const void *ximg, const float *xscale,
                         const float *xnorm, int64_t n, float *qscale, float *qres, const float *qnorm, void *qimg,
                         float *part_d, int *part_i, int64_t nw, hipStream_t st) {
    HIPANN_REQUIRE(nq >= 1 && nq <= flat_i8_scan_max_nq() && n >= 1 && nw >= 4 && nw % 4 == 0, "flat_i8_scan: shape");
    const int nk = flat_i8_nk(d);
    launch_i8_row_scale(Q, nq, d, qscale, qres, st);
    const int64_t units = nq * nk * 4;
    hipLaunchKernelGGL(i8_query_units, dim3((unsigned)ceil_div(units, 256)), dim3(256), 0, st, Q, qscale, nq, d, nk,
                       static_cast<uint4 *>(qimg));
    const int64_t ngroups = (n + 63) / 64;
    const int64_t gpw = ceil_div(ngroups, nw);
    const size_t smem = (size_t)nq * nk * 4 * sizeof(uint4);
    HIPANN_REQUIRE(smem <= 64 * 1024, "flat_i8_scan: query units exceed LDS");
    dim3 grid((unsigned)ceil_div(nw, 4)), block(256);
    const uint4 *qa = static_cast<const uint4 *>(qimg), *xa = static_cast<const uint4 *>(ximg);
#define I8S_CASE(NQV)                                                                                                  \
    case NQV:                                                                                                          \
        if (metric == kIP) hipLaunchKernelGGL((flat_i8_scan<NQV, true>), grid, block, smem, st, qa, qscale, qnorm, xa, \
                                              xscale, xnorm, n, nk, gpw, part_d, part_i);                              \
        else hipLaunchKernelGGL((flat_i8_scan<NQV, false>), grid, block, smem, st, qa, qscale, qnorm, xa, xscale,      \
                                xnorm, n, nk, gpw, part_d, part_i);                                                    \
        break;
    switch ((int)nq) {
        I8S_CASE(1) I8S_CASE(2) I8S_CASE(3) I8S_CASE(4) I8S_CASE(5) I8S_CASE(6) I8S_CASE(7) I8S_CASE(8) I8S_CASE(9)
        I8S_CASE(10) I8S_CASE(11) I8S_CASE(12) I8S_CASE(13) I8S_CASE(14) I8S_CASE(15) I8S_CASE(16)
        default: throw HipError("flat_i8_scan: nq");
    }
#undef I8S_CASE
    HIPANN_CHECK(hipGetLastError());
}
void launch_flat_i8_group_merge(const float *pd, const int *pi, int nw, int nq, int ngroup, float *od, int *oi,
                                hipStream_t st) {
    const int per = (int)ceil_div(nw, ngroup);
    const int64_t items = (int64_t)ngroup * nq;
    hipLaunchKernelGGL(flat_i8_group_merge, dim3((unsigned)ceil_div(items, 4)), dim3(256), 0, st, pd, pi, nw, nq, per,
                       ngroup, od, oi);
    HIPANN_CHECK(hipGetLastError());
}


void launch_flat_bf16_k64(const void *qimg, const float *qn, int64_t nq, const void *ximg, const float *xn, int64_t N,
                          int nk, int metric, int nqt, int nsplit, int64_t tiles_per_split, int64_t tile_begin,
                          int64_t tile_end, const float *bound, float *cand_d, int *cand_i, int *cand_n, int cap,
                          bool resume, bool keys, hipStream_t st, const float *qscale, const float *xscale) {
    HIPANN_REQUIRE(nk % 2 == 0 && cand_d && (keys || (bound && cand_i && cand_n && cap > 0)),
                   "flat_bf16_k64: bad arguments");
    HIPANN_REQUIRE(!qscale == !xscale, "flat_bf16_k64: int8 needs both scales");
    HIPANN_REQUIRE((int64_t)nqt * nsplit < 0x7fffffff, "grid too large");
    // (r05, measured and dropped: a 4-wave 512-register variant — 64 queries per wave, half the LDS reads per MFMA —
    // 9.93 vs 8.22 ms at 10M, its accumulators shuffled between AGPRs and VGPRs; a tile loop whose first K-step starts
    // from a zero C operand instead of resetting the accumulators — 43 spills, 10.75 vs 7.71 ms)
    dim3 grid((unsigned)(nqt * nsplit)), block(64 * K64Geom<2>::W);
    const k64_u32x4 *qa = static_cast<const k64_u32x4 *>(qimg);
    const k64_u32x4 *xa = static_cast<const k64_u32x4 *>(ximg);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, K64_LDS, st, qa, qn, nq, xa, xn, N, nk, nqt, nsplit, tiles_per_split,
                           tile_begin, tile_end, bound, cand_d, cand_i, cand_n, cap, resume ? 1 : 0, qscale, xscale);
    };
    // HIPANN_K64_STAGGER=1 (A/B, measured and rejected in r06): the staggered schedule (STAG above).  Same-box A/B,
    // alternating: 10M x 768 kernel 7.86-7.92 → 9.08-9.10 ms, C2 1.00 → 1.23, C5 9.69 → 11.12 (with the epilogue at
    // s_setprio 0 under the partner's MFMAs: no better) — the default keeps every wave on the same K-step.  It needs
    // ≥ 3 K-steps per tile (the tile's norms are loaded two K-steps before its epilogue).
    static const bool stag_env = [] { const char *e = std::getenv("HIPANN_K64_STAGGER"); return e && std::atoi(e); }();
    const bool stag = stag_env && nk / 2 >= 3;
    if (qscale) {
        if (keys) {
            if (metric == kL2) go(flat_bf16_k64<true, true, true>);
            else go(flat_bf16_k64<false, true, true>);
        } else if (stag) {
            if (metric == kL2) go(flat_bf16_k64<true, false, true, 2, true>);
            else go(flat_bf16_k64<false, false, true, 2, true>);
        } else {
            if (metric == kL2) go(flat_bf16_k64<true, false, true>);
            else go(flat_bf16_k64<false, false, true>);
        }
    } else if (keys) {
        if (metric == kL2) go(flat_bf16_k64<true, true>);
        else go(flat_bf16_k64<false, true>);
    } else {
        if (metric == kL2) go(flat_bf16_k64<true, false>);
        else go(flat_bf16_k64<false, false>);
    }
    HIPANN_CHECK(hipGetLastError());
}

// HIPANN_FLAT_CAND_NARROW=0 (A/B): the one-wave-per-query wave-list kernels
static bool cand_narrow_on(int k) {
    static const bool env = [] { const char *e = std::getenv("HIPANN_FLAT_CAND_NARROW"); return !e || std::atoi(e); }();
    return env && k <= 64;
}

void launch_flat_cand_bound(const float *cand_d, const int *cand_n, int nsplit, int cap, int64_t nq, int k,
                            float *bound, hipStream_t st) {
    if (nq <= 0) return;
    if (cand_narrow_on(k))
        hipLaunchKernelGGL(flat_cand_bound_nw, dim3((unsigned)nq), dim3(256), 0, st, cand_d, cand_n, nsplit, cap, nq, k,
                           bound);
    else
        hipLaunchKernelGGL(flat_cand_bound, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, cand_d, cand_n, nsplit,
                           cap, nq, k, bound);
    HIPANN_CHECK(hipGetLastError());
}

void launch_flat_cand_select(const float *cand_d, const int *cand_i, const int *cand_n, int nsplit, int cap, int64_t nq,
                             int k, float *out_d, int *out_i, int *nflag, int *flagged, hipStream_t st) {
    if (nq <= 0) return;
    if (cand_narrow_on(k))
        hipLaunchKernelGGL(flat_cand_select_nw, dim3((unsigned)nq), dim3(256), 0, st, cand_d, cand_i, cand_n, nsplit, cap,
                           nq, k, out_d, out_i, nflag, flagged);
    else
        hipLaunchKernelGGL(flat_cand_select, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, cand_d, cand_i, cand_n,
                           nsplit, cap, nq, k, out_d, out_i, nflag, flagged);
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann

// test hook (tests/test_abi.py): the small-batch int8 scan's wave count for an n-row table — a whole number of
// 4-wave blocks, so the launched grid never writes past the nw·nq·64 part buffers (no device needed)
extern "C" int64_t hipann_debug_flat_i8_scan_waves(int64_t n) { return hipann::flat_i8_scan_waves(n); }
