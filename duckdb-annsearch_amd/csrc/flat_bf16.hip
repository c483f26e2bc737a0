// flat_bf16.hip — Flat exact form on the plain bf16 matrix cores (form kFlatBf16Exact, the default).
//
// Replaces the GEMM + select half of MetalIndexFlat::search (faiss-metal/src/MetalIndexFlat.mm:294-369;
// MetalDistance.mm:107-288 simdgroup_gemm_l2_fused, MetalSelect.mm:31-74 warp/block select) for
// nq >= 20 (FAISS's BLAS path).  One q·x product per element instead of the split forms' three:
//
//   * the database is converted ONCE (at the first search after an add) into a tiled bf16 image, and
//     every batch's queries into the same layout: tile of R rows, chunk of 32 dims = R·4 units of 16 B,
//     unit b16_slot(c, row) = dims 8c..8c+7 of the row, XOR-swizzled so that the 16-B fragment reads of
//     v_mfma_f32_32x32x16_bf16 (16-lane groups of 16 distinct rows) and the linear staging writes are
//     bank-conflict free.  A chunk of a tile is 16 KB of consecutive HBM: the block copies it with one
//     coalesced 16-B load per thread per unit, no conversion in the loop;
//   * block = W waves, tile = 32W queries × 256 database rows; A (queries) and B (rows) chunks
//     double-buffered in LDS, one barrier per chunk; wave w owns queries [32w, 32w+32) × all 256 rows
//     (8 accumulators of 32×32), so a query's candidates never leave its wave;
//   * the epilogue (once per tile) filters keys straight from the accumulators: 2·ip − ‖x‖² ≥
//     ‖q‖² − thr is one fma + one compare per element (key = ‖q‖² + ‖x‖² − 2·ip, thr = the query's
//     k-th kept key; IP: 2·ip ≥ −2·thr); a ballot per accumulator row sends the rare passing rows to
//     the WaveList insert (exact keys, (key, row) order).  The filter's rounding (a few ulps of the
//     key magnitudes) is covered by the rerank bound's margin (below);
//   * output: the k best (key, row) per (database split, query), query-major, for ivf_rerank_topk.
//
// Exactness (ivf_rerank_topk, shared with the IVF exact form): the 32 best scan keys per (split, query)
// are merged to 32, recomputed in the fp32 direct form and ordered by (distance, label).  The scan key of
// any row differs from its fp32 distance by at most the Cauchy-Schwarz bound of the bf16 rounding,
// |q̂·x̂ − q·x| ≤ ‖q‖·‖x̂−x‖ + ‖q̂−q‖·‖x̂‖, with ‖x̂−x‖ ≤ rxmax (the largest row residual, measured when the
// image is built) and this query's own residual, plus the fp32 accumulation and rounding terms (the
// kernel's comment).  For U(−1,1) rows at d = 768 that is ≈1.3 against a ≈5 gap between the 10th and 32nd
// distances of 10M rows; a query whose k-th exact distance is not below K₃₂ − E re-runs on the 3-term
// split form.
#include "runtime.hpp"
#include "wave_topk.hpp"

#include <cstdlib>
#include <type_traits>
#include <utility>

namespace hipann {

typedef __bf16 b16x8 __attribute__((ext_vector_type(8)));
typedef float b16_f32x8 __attribute__((ext_vector_type(8)));
typedef float b16_f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned b16_u32x4 __attribute__((ext_vector_type(4)));  // 16-B unit (native vector: stays in VGPRs)

constexpr int B16_TN = 256;  // database rows per tile
constexpr int B16_KC = 32;   // dims per chunk

__host__ __device__ inline int b16_nk(int d) { return (d + B16_KC - 1) / B16_KC; }
// 16-B unit of (group c, row) in a chunk image of R rows
__device__ __forceinline__ int b16_slot(int c, int row, int R) { return c * R + (row ^ (c << 1)); }

// Tiled bf16 image of an n × d fp32 matrix, tiles of R rows: unit u = ((t·nk + kc)·4 + c)·R + (row ^ 2c)
// holds RNE bf16 of dims kc·32 + 8c .. +7 of row t·R + row (zero past n / d).  One thread per unit.
__global__ void __launch_bounds__(256) b16_tile_rows(const float *__restrict__ X, int64_t n, int d, int R, int nk,
                                                     int64_t total, uint4 *__restrict__ out) {
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
    const int dim0 = kc * B16_KC + 8 * c;
    b16_f32x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (grow < n && dim0 + i < d) ? X[grow * (int64_t)d + dim0 + i] : 0.f;
    const b16x8 b = __builtin_convertvector(v, b16x8);
    out[u] = __builtin_bit_cast(uint4, b);
}

// ‖bf16(x) − x‖² per row (one wave per row): the largest is the rerank bound's row term.
__global__ void __launch_bounds__(256) b16_row_residual2(const float *__restrict__ X, int64_t n, int d,
                                                         float *__restrict__ out) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    const float *x = X + row * (int64_t)d;
    float s = 0.f;
    for (int e = lane; e < d; e += 64) {
        const float r = x[e] - (float)(__bf16)x[e];
        s = fmaf(r, r, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) out[row] = s;
}

// Epilogue of one tile: acc[j] = q·x of query rows (r&3) + 8(r>>2) + 4h (+ 32·wave) and database row
// x0 + 32j + (lane & 31).  cth[r] = ‖q‖² − thr (L2) or −2·thr (IP); xnv[j] = ‖x‖² (L2) or 0, +inf past N.
// ‖q‖² of the lane's query row r is read from qnorm (L2-resident) on the slow path only, which keeps the
// main loop's registers for deeper LDS fragment prefetch.
template <bool L2M>
__device__ __forceinline__ void b16_epilogue(const b16_f32x16 (&acc)[8], float (&cth)[16],
                                             const float *__restrict__ qnorm, int64_t qrow0, int64_t nq,
                                             const float (&xnv)[8], int64_t x0, int64_t N, float *__restrict__ Ld,
                                             int *__restrict__ Li, int k, int wave, int lane) {
    const int l31 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) any |= fmaf(2.f, acc[j][r], -xnv[j]) >= cth[r];
        const unsigned long long m = __ballot(any);
        if (m == 0ull) continue;
        // slow path (rare after the first tiles): each half of the wave is one query
        const int64_t qr = qrow0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float qnr = (L2M && qr < nq) ? qnorm[qr] : 0.f;
        float key[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float kv;
            if (L2M) {
                kv = fmaf(-2.f, acc[j][r], qnr + xnv[j]);
                kv = kv < 0.f ? 0.f : kv;
            } else {
                kv = -acc[j][r];
            }
            key[j] = x0 + 32 * j + l31 < N ? kv : __builtin_inff();
        }
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            if (((m >> (32 * hh)) & 0xffffffffull) == 0ull) continue;
            const int ql = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const int src = 32 * hh + l31;
            WaveList<1, int> L;
            L.d[0] = lane < k ? Ld[ql * k + lane] : __builtin_inff();
            L.id[0] = lane < k ? Li[ql * k + lane] : 0x7fffffff;
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                const float c0 = __shfl(key[2 * o], src), c1 = __shfl(key[2 * o + 1], src);
                const float v = lane < 32 ? c0 : c1;
                const int64_t col = x0 + 32 * (2 * o + h) + l31;
                L.offer(v, col < N ? (int)col : 0x7fffffff, k - 1);
            }
            if (lane < k) {
                Ld[ql * k + lane] = L.d[0];
                Li[ql * k + lane] = L.id[0];
            }
            const float nt = readlane_f(L.d[0], k - 1);
            if (h == hh) cth[r] = L2M ? qnr - nt : -2.f * nt;
        }
    }
}

typedef __attribute__((address_space(3))) void b16_lds_void;

template <int N>
__device__ __forceinline__ void b16_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// RA (register A): each wave's query fragments (2 × 16 B per lane per chunk — no other wave reads them) come
// straight from the L2-resident query image into a 3-deep register ring instead of through LDS, so the
// LDS-DMA fill carries only the shared database tile: 16 KB per 32-dim chunk instead of 32 KB (the fill
// rate, ≈6 TB/s chip-wide, is what bounds this kernel at 128 FLOP/B).
template <bool L2M, int W, bool RA, int NB = 3>
__global__ void __launch_bounds__(64 * W, 1)
flat_bf16_topk(const b16_u32x4 *__restrict__ Qt, const float *__restrict__ qnorm, int64_t nq,
               const b16_u32x4 *__restrict__ Xt,
               const float *__restrict__ xnorm, int64_t N, int nk, int k, int nqt, int nsplit,
               int64_t tiles_per_split, float *__restrict__ part_d, int *__restrict__ part_i,
               const float *__restrict__ seed) {
    constexpr int QM = 32 * W;
    constexpr int AU = QM * 4, BU = B16_TN * 4;  // 16-B units per chunk image
    constexpr int SU = RA ? BU : AU + BU;        // units per LDS stage
    // NB stages: chunks g+1 .. g+NB−1 in flight while chunk g is read (NB − 1 chunk times to cover the
    // LDS-DMA issue → landed latency, ≈1.1 µs)
    static_assert(NB >= 3 && NB <= 6, "stages");
    constexpr int IA = AU / 64 / W, IB = BU / 64 / W;  // global_load_lds (1 KiB each) per wave per chunk
    constexpr int NI = RA ? IB + 2 : IA + IB;   // vector-memory ops per wave per chunk
    static_assert(IA * 64 * W == AU && IB * 64 * W == BU, "chunk images must split evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) b16_u32x4 smem_b16[];
    float *Ld = reinterpret_cast<float *>(smem_b16 + NB * SU);  // [QM][k]
    int *Li = reinterpret_cast<int *>(Ld + QM * k);

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * QM;
    const int64_t ntiles = ceil_div(N, B16_TN);
    const int64_t t0 = (int64_t)split * tiles_per_split;
    const int64_t t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;
    const int64_t G = t1 > t0 ? (t1 - t0) * nk : 0;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int l31 = lane & 31, h = lane >> 5;

    // seed (optional): per query an upper bound T_q of its k-th best scan key (the k-th best over a sample of
    // rows, flat_bf16_seed).  The list starts as k copies of (T_q, pad): only keys ≤ T_q are admitted, and
    // the pads never reach the rerank (their row id is out of range)
    for (int e = tid; e < QM * k; e += 64 * W) {
        const int64_t q = q0 + e / k;
        Ld[e] = seed && q < nq ? seed[q] : __builtin_inff();
        Li[e] = 0x7fffffff;
    }
    float cth[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float qn = (L2M && q < nq) ? qnorm[q] : 0.f;
        const float thr = q < nq ? (seed ? seed[q] : __builtin_inff()) : -__builtin_inff();  // −inf: rows past nq
        cth[r] = L2M ? qn - thr : -2.f * thr;
    }

    // chunk g = (t − t0)·nk + kc: query chunk kc and database chunk t·nk + kc (a split's database chunks are
    // consecutive in the image).  LDS-DMA (global_load_lds_dwordx4): each wave copies its share of the two
    // images, 1 KiB per instruction, into stage g % NB — lane-linear, the swizzle is in the images themselves.
    const b16_u32x4 *Qb = Qt + (int64_t)qt * nk * AU + lane;
    const b16_u32x4 *Xb = Xt + t0 * nk * BU + lane;
    int kc_issue = 0;
    // RA: this lane's fragment of query chunk kc, k-step s (c = 2s + h), read from the image directly
    const b16_u32x4 *Qw = Qt + (int64_t)qt * nk * AU + 32 * wave;
    b16_u32x4 ar[NB][2];  // RA register ring (slot = chunk % NB, compile-time after unrolling)
    auto issue = [&](int64_t g, int stage, auto slot_c) {
        constexpr int SL = decltype(slot_c)::value;
        b16_u32x4 *dst = smem_b16 + stage * SU;
        if constexpr (RA) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int c = 2 * s2 + h;
                ar[SL][s2] = Qw[(int64_t)kc_issue * AU + c * QM + (l31 ^ (c << 1))];
            }
        } else {
#pragma unroll
            for (int i = 0; i < IA; ++i) {
                const int inst = wave * IA + i;
                __builtin_amdgcn_global_load_lds((const void *)(Qb + (int64_t)kc_issue * AU + inst * 64),
                                                 (b16_lds_void *)(dst + inst * 64), 16, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int inst = wave * IB + i;
            __builtin_amdgcn_global_load_lds((const void *)(Xb + g * BU + inst * 64),
                                             (b16_lds_void *)(dst + (RA ? 0 : AU) + inst * 64), 16, 0, 0);
        }
        kc_issue = kc_issue + 1 < nk ? kc_issue + 1 : 0;
    };

    b16_f32x16 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    __syncthreads();  // list initialisation
    using I0 = std::integral_constant<int, 0>;
    if (RA && G > 0) {  // the ring starts full (past the end: the last chunk again)
        [&]<int... P>(std::integer_sequence<int, P...>) {
            (issue(P < G ? P : G - 1, P, std::integral_constant<int, P>{}), ...);
        }(std::make_integer_sequence<int, NB - 1>{});
    } else {
        [&]<int... P>(std::integer_sequence<int, P...>) {
            ((P < G ? issue(P, P, std::integral_constant<int, P>{}) : void()), ...);
        }(std::make_integer_sequence<int, NB - 1>{});
    }

    int kc = 0, stage = 0;
    int64_t t = t0;
    // one chunk; SL = g % NB (RA's register slot; the loop below is unrolled by NB)
    auto body = [&](int64_t g, auto slot_c) {
        constexpr int SL = decltype(slot_c)::value;
        // retire this wave's copies of chunk g (chunk g+1's stay in flight), finish this wave's reads of the
        // stage about to be refilled, then one barrier: every wave's chunk-g copies have landed and nobody
        // still reads stage (g+2) % NB = (g−1) % NB
        // RA: the issue is unconditional (past the end it re-reads the last chunk into a free stage), so every
        // iteration has the same count of vector-memory ops and the compiler's own waits stay exact
        if (RA) b16_wait_vm<NI * (NB - 2)>();
        else if (g + NB - 2 < G) b16_wait_vm<NI * (NB - 2)>();
        else b16_wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int st_next = stage == 0 ? NB - 1 : stage - 1;  // (stage + NB − 1) % NB: chunk g−1's, now free
        if (RA) issue(g + NB - 1 < G ? g + NB - 1 : G - 1, st_next, std::integral_constant<int, (SL + NB - 1) % NB>{});
        else if (g + NB - 1 < G) issue(g + NB - 1, st_next, std::integral_constant<int, (SL + NB - 1) % NB>{});
        const b16_u32x4 *Ab = smem_b16 + stage * SU;
        const b16_u32x4 *Bb = Ab + (RA ? 0 : AU);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 2 * s + h;
            // every fragment of this k-step read before its MFMAs: one LDS wait per 8 MFMAs instead of
            // one per MFMA
            // b16_slot(c, 32·j + l31, R) = c·R + 32·j + (l31 ^ 2c) (the swizzle stays inside the low 5 bits):
            // one base per c, the j offsets are immediates
            const int lx = l31 ^ (c << 1);
            const b16x8 a = RA ? __builtin_bit_cast(b16x8, ar[SL][s])
                               : __builtin_bit_cast(b16x8, Ab[c * QM + 32 * wave + lx]);
            const b16_u32x4 *Bc = Bb + c * B16_TN + lx;
            b16x8 bf[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) bf[j] = __builtin_bit_cast(b16x8, Bc[32 * j]);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf[j], acc[j], 0, 0, 0);
            // schedule: three LDS reads ahead, then one MFMA per read — each fragment is read two MFMAs
            // (≥ 64 cycles) before its use instead of waiting on a read issued just before
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
        }
        stage = stage + 1 < NB ? stage + 1 : 0;
        if (++kc == nk) {
            kc = 0;
            const int64_t x0 = t * B16_TN;
            float xnv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int64_t x = x0 + 32 * j + l31;
                xnv[j] = x < N ? (L2M ? xnorm[x] : 0.f) : __builtin_inff();
            }
            b16_epilogue<L2M>(acc, cth, qnorm, q0 + 32 * wave, nq, xnv, x0, N, Ld, Li, k, wave, lane);
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
            ++t;
        }
    };
    if constexpr (RA) {
        for (int64_t g = 0; g < G; g += NB) {
            [&]<int... P>(std::integer_sequence<int, P...>) {
                ((g + P < G ? body(g + P, std::integral_constant<int, P>{}) : void()), ...);
            }(std::make_integer_sequence<int, NB>{});
        }
        b16_wait_vm<0>();  // no LDS-DMA copy may land after the block's LDS is handed to the next block
    } else {
        for (int64_t g = 0; g < G; ++g) body(g, I0{});
    }
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

// Seed thresholds: per query the k-th smallest key of its nsplit partial lists (query-major [q][split][k]),
// raised by a few ulps (the main pass recomputes those sample rows' keys bit-identically; the margin only
// guards the ≥ k rows with key ≤ T_q that make the rerank's K_k ≤ T_q).  One wave per query.
__global__ void __launch_bounds__(256) flat_bf16_seed(const float *__restrict__ pd, int nsplit, int64_t nq, int k,
                                                      float *__restrict__ seed) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<1, int> L;
    L.init();
    const int64_t total = (int64_t)nsplit * k;
    for (int64_t c0 = 0; c0 < total; c0 += 64) {
        const int64_t c = c0 + lane;
        const float v = c < total ? pd[q * total + c] : __builtin_inff();
        L.offer(v, (int)lane, k - 1);
    }
    if (lane == 0) {
        const float t = readlane_f(L.d[0], k - 1);
        seed[q] = t == __builtin_inff() ? t : fmaxf(t * (1.f + 0x1p-20f), t + 0x1p-100f);
    }
}

// ------------------------------------------------------------------------------------------------
constexpr int kB16StagesDefault = 4;  // 10M x 768: 19.16 (3) / 18.68 (4) / 19.06 (5) ms
int flat_bf16_waves(int64_t nq) { return nq >= 256 ? 8 : nq >= 128 ? 4 : 2; }
int flat_bf16_tile_rows() { return B16_TN; }
// the largest list length k (≤ 64) of flat_bf16_topk's LDS lists at this batch size (its launcher's LDS check)
int flat_bf16_topk_kmax(int64_t nq) {
    const int QM = 32 * flat_bf16_waves(nq);
    int k = 64;
    while (k > 1 && (size_t)3 * (QM * 4 + B16_TN * 4) * 16 + (size_t)QM * k * 8 > 160 * 1024) --k;
    return k;
}

size_t flat_bf16_img_bytes(int64_t n, int d, int R) {
    return (size_t)ceil_div(std::max<int64_t>(n, 1), R) * b16_nk(d) * R * 4 * 16;
}

void launch_b16_tile_rows(const float *X, int64_t n, int d, int R, void *out, hipStream_t st) {
    const int nk = b16_nk(d);
    const int64_t total = ceil_div(std::max<int64_t>(n, 1), R) * nk * R * 4;
    hipLaunchKernelGGL(b16_tile_rows, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, st, X, n, d, R, nk, total,
                       static_cast<uint4 *>(out));
    HIPANN_CHECK(hipGetLastError());
}

void launch_b16_row_residual2(const float *X, int64_t n, int d, float *out, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(b16_row_residual2, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, X, n, d, out);
    HIPANN_CHECK(hipGetLastError());
}

void launch_flat_bf16_seed(const float *pd, int nsplit, int64_t nq, int k, float *seed, hipStream_t st) {
    if (nq <= 0) return;
    hipLaunchKernelGGL(flat_bf16_seed, dim3((unsigned)ceil_div(nq, 4)), dim3(256), 0, st, pd, nsplit, nq, k, seed);
    HIPANN_CHECK(hipGetLastError());
}

// the bounded passes of flat_b16k64.hip apply to 256-query blocks over an even chunk count (HIPANN_B16_K64=0:
// one pass of the 32-dim list kernel below, A/B)
bool flat_bf16_resumable(int64_t nq, int d, int k) {
    static const bool k64 = [] { const char *e = std::getenv("HIPANN_B16_K64"); return !e || std::atoi(e); }();
    return k64 && flat_bf16_waves(nq) == 8 && flat_bf16_k64_supported(b16_nk(d), k);
}

void launch_flat_bf16_topk(const float *Q, const float *qn, int64_t nq, void *qimg, const void *ximg, const float *xn,
                           int64_t N, int d, int metric, int k, int nsplit, int64_t tiles_per_split, float *pd, int *pi,
                           const float *seed, bool image_ready, hipStream_t st) {
    const int W = flat_bf16_waves(nq);
    const int QM = 32 * W;
    const int nk = b16_nk(d);
    if (!image_ready) launch_b16_tile_rows(Q, nq, d, QM, qimg, st);
    const int nqt = (int)ceil_div(nq, QM);
    const size_t smem = (size_t)3 * (QM * 4 + B16_TN * 4) * 16 + (size_t)QM * k * 8;
    HIPANN_REQUIRE(smem <= 160 * 1024, "k too large for the bf16 Flat kernel");
    HIPANN_REQUIRE((int64_t)nqt * nsplit < 0x7fffffff, "grid too large");
    dim3 grid((unsigned)(nqt * nsplit)), block(64 * W);
    const b16_u32x4 *qa = static_cast<const b16_u32x4 *>(qimg);
    const b16_u32x4 *xa = static_cast<const b16_u32x4 *>(ximg);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, smem, st, qa, qn, nq, xa, xn, N, nk, k, nqt, nsplit, tiles_per_split, pd,
                           pi, seed);
    };
    static const bool ra = [] { const char *e = std::getenv("HIPANN_B16_RA"); return !e || std::atoi(e); }();
    // RA stages (HIPANN_B16_NB = 3..5, A/B): LDS-DMA chunks in flight = NB − 1
    static const int nb = [] { const char *e = std::getenv("HIPANN_B16_NB"); const int v = e ? std::atoi(e) : 0;
                               return v >= 3 && v <= 5 ? v : kB16StagesDefault; }();
    const size_t smem_ra = (size_t)nb * (B16_TN * 4) * 16 + (size_t)QM * k * 8;
    if (ra && W == 8 && smem_ra <= 160 * 1024) {
        auto go_ra = [&](auto kern) {
            hipLaunchKernelGGL(kern, grid, block, smem_ra, st, qa, qn, nq, xa, xn, N, nk, k, nqt, nsplit, tiles_per_split,
                               pd, pi, seed);
        };
        if (metric == kL2) {
            if (nb == 3) go_ra(flat_bf16_topk<true, 8, true, 3>);
            else if (nb == 4) go_ra(flat_bf16_topk<true, 8, true, 4>);
            else go_ra(flat_bf16_topk<true, 8, true, 5>);
        } else {
            if (nb == 3) go_ra(flat_bf16_topk<false, 8, true, 3>);
            else if (nb == 4) go_ra(flat_bf16_topk<false, 8, true, 4>);
            else go_ra(flat_bf16_topk<false, 8, true, 5>);
        }
    } else if (metric == kL2) {
        if (W == 8) go(flat_bf16_topk<true, 8, false>);
        else if (W == 4) go(flat_bf16_topk<true, 4, false>);
        else go(flat_bf16_topk<true, 2, false>);
    } else {
        if (W == 8) go(flat_bf16_topk<false, 8, false>);
        else if (W == 4) go(flat_bf16_topk<false, 4, false>);
        else go(flat_bf16_topk<false, 2, false>);
    }
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
