// flat_b16k64.hip — the Flat bf16 filter scan (form kFlatBf16Exact) with 64-dim K-steps on
// v_mfma_f32_16x16x32_bf16.
//
// Same job, images and output as flat_bf16_topk (flat_bf16.hip: MetalIndexFlat::search's GEMM + select for
// nq >= 20, faiss-metal/src/MetalIndexFlat.mm:294-369): per (database split, query) the k best scan keys
// of one bf16 product per element, as the filter of the exact fp32 rerank (ivf_rerank_topk).  What
// changes is the main loop, after the 256² GEMM recipe of cdna_hip_programming.md §5:
//   * K-step = 64 dims (two 32-dim image chunks, consecutive in the tiled image): one barrier and one
//     counted vmcnt per 64 MFMAs per wave instead of per 16 — BK 32 → 64 is the first lever of that recipe;
//   * v_mfma_f32_16x16x32_bf16 (16-cycle issue; the chip holds a higher clock on it than on the 32×32×16
//     shape under load, MI355X_MICROARCH.md 'DVFS give-back' item 7): wave w owns queries [32w, 32w+32) ×
//     all 256 rows of the tile = 2 × 16 accumulators of 16 × 16;
//   * the database tile streams by LDS-DMA into 3 stages of 32 KB (K-steps g+1 and g+2 in flight), the
//     query fragments straight into a 2-deep register ring (each wave reads only its own queries); the
//     per-query top-k lists stay in LDS: 3 × 32 KB + 256 × k × 8 B = 160 KiB at k = 32.
// Keys, lists and the epilogue's filter (2·ip − ‖x‖² ≥ ‖q‖² − thr) are those of flat_bf16_topk; only the
// fp32 accumulation order of the bf16 products differs, which the rerank bound covers (any order of d
// exact products: the (d + 8)·2⁻²⁴ term).
#include "runtime.hpp"
#include "wave_topk.hpp"

#include <cstdlib>
#include <type_traits>
#include <utility>

namespace hipann {

typedef __bf16 k64_b16x8 __attribute__((ext_vector_type(8)));
typedef float k64_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned k64_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void k64_lds_void;

constexpr int K64_TN = 256;               // database rows per tile
constexpr int K64_QM = 256;               // queries per block (8 waves × 32)
constexpr int K64_W = 8;
constexpr int K64_NB = 3;                 // LDS stages (K-steps g+1, g+2 in flight while g is read)
constexpr int K64_BU = K64_TN * 4;        // 16-B units of one 32-dim chunk of a database tile
constexpr int K64_SU = 2 * K64_BU;        // units per stage (one 64-dim K-step): 32 KB
constexpr int K64_PIECES = K64_SU / 64 / K64_W;  // 1-KiB LDS-DMA pieces per wave per K-step
static_assert(K64_PIECES * 64 * K64_W == K64_SU, "pieces split evenly");

template <int N>
__device__ __forceinline__ void k64_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue of one tile.  On entry acc[mb][jb][i] = s = 2·q·x − ‖x‖² (L2; 2·q·x for IP, −inf past N) of query
// 32·wave + 16·mb + 4·(lane >> 4) + i and database row x0 + 16·jb + (lane & 15); a row passes the query's
// bound when s ≥ cth = ‖q‖² − thr (L2) or −2·thr (IP) — cth[mb][i] is the lane's own query's (its 16-lane
// group).  Rare passing rows go through the query's LDS list (one WaveList of k per query, offered 64
// candidates per round) with key = ‖q‖² − s (L2, clamped at 0) or −s/2 = −q·x (IP): +inf past N.
template <bool L2M, int MB, int I>
__device__ __forceinline__ void k64_epilogue_row(const k64_f32x4 (&acc)[2][16], float (&cth)[2][4],
                                                 const float *__restrict__ qnorm, int64_t q0wave, int64_t nq,
                                                 int64_t x0, int64_t N, float *__restrict__ Ld,
                                                 int *__restrict__ Li, int k, int wave, int lane) {
    const int m16 = lane & 15, g4 = lane >> 4;
    bool any = false;
#pragma unroll
    for (int jb = 0; jb < 16; ++jb) any |= acc[MB][jb][I] >= cth[MB][I];
    const unsigned long long m = __ballot(any);
    if (m == 0ull) return;
#pragma unroll 1
    for (int fq = 0; fq < 4; ++fq) {
        if (((m >> (16 * fq)) & 0xffffull) == 0ull) continue;
        const int ql = 32 * wave + 16 * MB + 4 * fq + I;
        const int64_t qr = q0wave + 16 * MB + 4 * fq + I;  // wave-uniform
        const float qnr = (L2M && qr < nq) ? qnorm[qr] : 0.f;
        WaveList<1, int> L;
        L.d[0] = lane < k ? Ld[ql * k + lane] : __builtin_inff();
        L.id[0] = lane < k ? Li[ql * k + lane] : 0x7fffffff;
        const int src = 16 * fq + m16;  // the lanes of query fq hold its 256 scores (16 per lane)
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            const float c0 = __shfl(acc[MB][4 * o + 0][I], src), c1 = __shfl(acc[MB][4 * o + 1][I], src);
            const float c2 = __shfl(acc[MB][4 * o + 2][I], src), c3 = __shfl(acc[MB][4 * o + 3][I], src);
            const float sv = g4 == 0 ? c0 : g4 == 1 ? c1 : g4 == 2 ? c2 : c3;
            float key;
            if (L2M) {
                key = qnr - sv;
                key = key < 0.f ? 0.f : key;
            } else {
                key = -0.5f * sv;
            }
            const int64_t col = x0 + 16 * (4 * o + g4) + m16;
            L.offer(key, col < N ? (int)col : 0x7fffffff, k - 1);
        }
        if (lane < k) {
            Ld[ql * k + lane] = L.d[0];
            Li[ql * k + lane] = L.id[0];
        }
        const float nt = readlane_f(L.d[0], k - 1);
        if (g4 == fq) cth[MB][I] = L2M ? qnr - nt : -2.f * nt;
    }
}

template <bool L2M>
__device__ __forceinline__ void k64_epilogue(k64_f32x4 (&acc)[2][16], float (&cth)[2][4],
                                             const float *__restrict__ qnorm, int64_t q0wave, int64_t nq,
                                             const float *__restrict__ xnorm, int64_t x0, int64_t N,
                                             float *__restrict__ Ld, int *__restrict__ Li, int k, int wave,
                                             int lane) {
    const int m16 = lane & 15;
    // s = 2·q·x − ‖x‖² in place (the filter's left side; the key follows from it with one more rounding,
    // inside the rerank bound's (d + 8)·2⁻²⁴ term): no ‖x‖² registers live through the list updates
#pragma unroll
    for (int jb = 0; jb < 16; ++jb) {
        const int64_t x = x0 + 16 * jb + m16;
        const float xv = x < N ? (L2M ? xnorm[x] : 0.f) : __builtin_inff();
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[mb][jb][i] = fmaf(2.f, acc[mb][jb][i], -xv);
    }
    [&]<int... P>(std::integer_sequence<int, P...>) {
        (k64_epilogue_row<L2M, P / 4, P % 4>(acc, cth, qnorm, q0wave, nq, x0, N, Ld, Li, k, wave, lane), ...);
    }(std::make_integer_sequence<int, 8>{});
}

template <bool L2M>
__global__ void __launch_bounds__(64 * K64_W, 1)
flat_bf16_k64(const k64_u32x4 *__restrict__ Qt, const float *__restrict__ qnorm, int64_t nq,
              const k64_u32x4 *__restrict__ Xt, const float *__restrict__ xnorm, int64_t N, int nk, int k, int nqt,
              int nsplit, int64_t tiles_per_split, float *__restrict__ part_d, int *__restrict__ part_i,
              const float *__restrict__ seed) {
    constexpr int NB = K64_NB;
    extern __shared__ __attribute__((aligned(16))) k64_u32x4 smem_k64[];
    float *Ld = reinterpret_cast<float *>(smem_k64 + NB * K64_SU);  // [QM][k]
    int *Li = reinterpret_cast<int *>(Ld + K64_QM * k);

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * K64_QM;
    const int64_t ntiles = ceil_div(N, K64_TN);
    const int64_t t0 = (int64_t)split * tiles_per_split;
    const int64_t t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;
    const int ns = nk >> 1;  // K-steps per tile (nk even)
    const int64_t G = t1 > t0 ? (t1 - t0) * ns : 0;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int m16 = lane & 15, g4 = lane >> 4;
    const int64_t q0w = q0 + 32 * wave + 4 * g4;  // + 16·mb + i: the lane's accumulator query rows
    const int64_t q0wave = q0 + 32 * __builtin_amdgcn_readfirstlane(wave);

    // seed (optional, as flat_bf16_topk): lists start at k copies of (T_q, pad)
    for (int e = tid; e < K64_QM * k; e += 64 * K64_W) {
        const int64_t q = q0 + e / k;
        Ld[e] = seed && q < nq ? seed[q] : __builtin_inff();
        Li[e] = 0x7fffffff;
    }
    float cth[2][4];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t q = q0w + 16 * mb + i;
            const float qn = (L2M && q < nq) ? qnorm[q] : 0.f;
            const float thr = q < nq ? (seed ? seed[q] : __builtin_inff()) : -__builtin_inff();
            cth[mb][i] = L2M ? qn - thr : -2.f * thr;
        }

    // K-step g = (t − t0)·ns + s covers image chunks 2s, 2s + 1 of tile t: 2·K64_BU consecutive units
    const k64_u32x4 *Xb = Xt + t0 * nk * K64_BU + lane;
    // the lane's query fragments: rows 32·wave + 16·mb + m16, unit c = g4 of each 32-dim chunk
    const k64_u32x4 *Qw = Qt + (int64_t)qt * nk * (K64_QM * 4) + g4 * K64_QM;
    const int qrow0 = (32 * wave + m16) ^ (g4 << 1), qrow1 = (32 * wave + 16 + m16) ^ (g4 << 1);
    // query fragments: a 2-deep register ring, K-step g+1's issued (before K-step g+2's tile pieces) while g
    // is computed, so at the top of K-step g only g+1's pieces may stay in flight
    int ks_a = 0;
    k64_u32x4 ar[2][2][2];  // [ring slot][chunk of the K-step][mb]
    auto issue_a = [&](auto slot_c) {
        constexpr int SL = decltype(slot_c)::value;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t kc = 2 * ks_a + h;
            ar[SL][h][0] = Qw[kc * (K64_QM * 4) + qrow0];
            ar[SL][h][1] = Qw[kc * (K64_QM * 4) + qrow1];
        }
        ks_a = ks_a + 1 < ns ? ks_a + 1 : 0;
    };
    auto issue_b = [&](int64_t g, int stage) {
        k64_u32x4 *dst = smem_k64 + stage * K64_SU;
#pragma unroll
        for (int i = 0; i < K64_PIECES; ++i) {
            const int inst = wave * K64_PIECES + i;
            __builtin_amdgcn_global_load_lds((const void *)(Xb + g * K64_SU + inst * 64),
                                             (k64_lds_void *)(dst + inst * 64), 16, 0, 0);
        }
    };

    k64_f32x4 acc[2][16];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int jb = 0; jb < 16; ++jb) acc[mb][jb] = (k64_f32x4){0.f, 0.f, 0.f, 0.f};
    __syncthreads();  // list initialisation
    if (G > 0) {  // A(0), B(0), B(1) (past the end: the last K-step again, never read)
        issue_a(std::integral_constant<int, 0>{});
        issue_b(0, 0);
        issue_b(G > 1 ? 1 : 0, 1);
    }

    int ks = 0, stage = 0;
    int64_t t = t0;
    auto body = [&](int64_t g, auto slot_c) {
        constexpr int SL = decltype(slot_c)::value;
        // K-step g landed (this wave's ops; B(g+1) stays in flight), every wave done reading the stage about
        // to be refilled (g−1's), one barrier; the issues are unconditional so the compiler's waits stay exact
        k64_wait_vm<K64_PIECES>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue_a(std::integral_constant<int, 1 - SL>{});
        issue_b(g + 2 < G ? g + 2 : G - 1, stage == 0 ? NB - 1 : stage - 1);
        const k64_u32x4 *Bb = smem_k64 + stage * K64_SU;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // B fragment of rows 16·jb + m16, unit c = g4: slot c·256 + 16·jb + (m16 ^ 2c)
            const k64_u32x4 *Bc = Bb + h * K64_BU + g4 * K64_TN + (m16 ^ (g4 << 1));
            const k64_b16x8 a0 = __builtin_bit_cast(k64_b16x8, ar[SL][h][0]);
            const k64_b16x8 a1 = __builtin_bit_cast(k64_b16x8, ar[SL][h][1]);
            k64_b16x8 bf[16];
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) bf[jb] = __builtin_bit_cast(k64_b16x8, Bc[16 * jb]);
#pragma unroll
            for (int jb = 0; jb < 16; ++jb) {
                acc[0][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[jb], acc[0][jb], 0, 0, 0);
                acc[1][jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[jb], acc[1][jb], 0, 0, 0);
            }
            // schedule (same region): four LDS reads ahead, then one read per MFMA pair
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int jb = 0; jb < 12; ++jb) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        }
        stage = stage + 1 < NB ? stage + 1 : 0;
        if (++ks == ns) {
            ks = 0;
            const int64_t x0 = t * K64_TN;
            k64_epilogue<L2M>(acc, cth, qnorm, q0wave, nq, xnorm, x0, N, Ld, Li, k, wave, lane);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int jb = 0; jb < 16; ++jb) acc[mb][jb] = (k64_f32x4){0.f, 0.f, 0.f, 0.f};
            ++t;
        }
    };
    for (int64_t g = 0; g < G; g += 2) {
        body(g, std::integral_constant<int, 0>{});
        if (g + 1 < G) body(g + 1, std::integral_constant<int, 1>{});
    }
    k64_wait_vm<0>();  // no LDS-DMA copy may land after the block's LDS is handed to the next block
    __syncthreads();
    // per-(split, query) lists, query-major (ivf_rerank_topk reads a query's lists contiguously)
    for (int r = 0; r < 32; ++r) {
        const int ql = 32 * wave + r;
        const int64_t q = q0 + ql;
        if (q < nq && lane < k) {
            const int64_t off = (q * nsplit + split) * k;
            part_d[off + lane] = Ld[ql * k + lane];
            part_i[off + lane] = Li[ql * k + lane];
        }
    }
}

// The K-step-64 kernel applies to 256-query blocks over an image with an even chunk count; the caller
// (launch_flat_bf16_topk) falls back to flat_bf16_topk otherwise.
bool flat_bf16_k64_supported(int nk, int k) {
    return nk % 2 == 0 && (size_t)K64_NB * K64_SU * 16 + (size_t)K64_QM * k * 8 <= 160 * 1024;
}

void launch_flat_bf16_k64(const void *qimg, const float *qn, int64_t nq, const void *ximg, const float *xn, int64_t N,
                          int nk, int metric, int k, int nqt, int nsplit, int64_t tiles_per_split, float *pd, int *pi,
                          const float *seed, hipStream_t st) {
    HIPANN_REQUIRE(flat_bf16_k64_supported(nk, k), "flat_bf16_k64: unsupported shape");
    const size_t smem = (size_t)K64_NB * K64_SU * 16 + (size_t)K64_QM * k * 8;
    dim3 grid((unsigned)(nqt * nsplit)), block(64 * K64_W);
    const k64_u32x4 *qa = static_cast<const k64_u32x4 *>(qimg);
    const k64_u32x4 *xa = static_cast<const k64_u32x4 *>(ximg);
    if (metric == kL2)
        hipLaunchKernelGGL(flat_bf16_k64<true>, grid, block, smem, st, qa, qn, nq, xa, xn, N, nk, k, nqt, nsplit,
                           tiles_per_split, pd, pi, seed);
    else
        hipLaunchKernelGGL(flat_bf16_k64<false>, grid, block, smem, st, qa, qn, nq, xa, xn, N, nk, k, nqt, nsplit,
                           tiles_per_split, pd, pi, seed);
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
