// flat_kernels.hip — Flat (brute-force) search kernels for gfx950.
//
// Replaces the faiss-metal Flat pipeline (MetalIndexFlat::search, MetalIndexFlat.mm:294-369):
//   l2_norm*.metal            → row_norms_f32
//   simdgroup_gemm*.metal + warp/block_select.metal (nq×N distance matrix, then select)
//                             → flat_gemm_topk: fp32 MFMA Q·Xᵀ with the L2 epilogue and a
//                               wave-distributed top-k fused in; the nq×N matrix never exists
//   fused_l2_topk.metal (small nq streaming scan)
//                             → flat_scan_topk: direct Σ(q−x)², HBM-bound
//   (host k-way merge)        → merge_parts_topk
//
// Distance forms follow FAISS CPU (the parity target, SURVEY §8a semantic contract):
//   nq <  20  → direct Σ(q−x)² (fvec_L2sqr)                      → flat_scan_topk
//   nq >= 20  → ‖q‖² + ‖x‖² − 2·q·x, clamped ≥ 0 (BLAS path)      → flat_gemm_topk
//   IP        → q·x, best = largest (selected as key = −q·x)
#include "common.hpp"
#include "wave_topk.hpp"

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <utility>

namespace hipann {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// ‖x‖² per row.  One wave per row, float4 loads when d % 4 == 0 (and 16-B aligned rows).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) row_norms_f32(const float *__restrict__ x, int64_t n, int d, int vec4,
                                                     float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const float *p = x + row * (int64_t)d;
    float s = 0.f;
    if (vec4) {
        const float4 *p4 = reinterpret_cast<const float4 *>(p);
        for (int j = lane; j < (d >> 2); j += 64) {
            float4 v = p4[j];
            s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
        }
    } else {
        for (int j = lane; j < d; j += 64) s = fmaf(p[j], p[j], s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) out[row] = s;
}

// ---------------------------------------------------------------------------------------------
// flat_gemm_topk — fp32 MFMA (v_mfma_f32_32x32x2_f32, exact f32 fma chain) tile GEMM with a fused
// distance epilogue and per-query top-k.  Block = 256 threads (4 waves), tile = 128 queries × 128
// database rows, K staged through LDS in chunks of 32 (double buffered, register staging).
//
// Grid: nqt × nsplit blocks, XCD-remapped so that the nqt query tiles of one database split run on
// the same XCD (they stream the same X rows: one HBM read, the rest L2 hits).  Each block walks the
// database tiles [t0, t1) of its split and keeps, per query row, a wave-distributed list of the 64
// best (key, row) pairs; at the end the first k go to part_d/part_i[split][q][0..k).
// ---------------------------------------------------------------------------------------------
constexpr int GBM = 128, GBN = 128, GBK = 32, GLD = GBK + 4;  // +4 floats: conflict-free ds_read_b128

template <bool VEC4>
__device__ __forceinline__ void gemm_stage_load(const float *__restrict__ base, int64_t row0, int64_t nrows,
                                                int d, int k0, float4 (&r)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int f = t + 256 * p;  // float4 index within the 128×32 tile
        const int row = f >> 3, c4 = f & 7;
        const int64_t grow = row0 + row;
        const int kk = k0 + 4 * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (grow < nrows) {
            const float *src = base + grow * (int64_t)d + kk;
            if (VEC4) {
                if (kk < d) v = *reinterpret_cast<const float4 *>(src);
            } else {
                if (kk + 0 < d) v.x = src[0];
                if (kk + 1 < d) v.y = src[1];
                if (kk + 2 < d) v.z = src[2];
                if (kk + 3 < d) v.w = src[3];
            }
        }
        r[p] = v;
    }
}

__device__ __forceinline__ void gemm_stage_store(float *__restrict__ lds, const float4 (&r)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int f = t + 256 * p;
        const int row = f >> 3, c4 = f & 7;
        *reinterpret_cast<float4 *>(lds + row * GLD + 4 * c4) = r[p];
    }
}

// WRITE = true: no selection — the epilogue writes the keys of every (query, row) pair of the
// tile to keys_out[q * ldk + row] (the k > 64 path selects from that matrix with rows_topk).
template <bool VEC4, bool WRITE = false>
__global__ void __launch_bounds__(256, 1)
flat_gemm_topk(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq,
               const float *__restrict__ X, const float *__restrict__ xnorm, int64_t N, int d, int metric,
               int k, int nqt, int nsplit, int64_t tiles_per_split, float *__restrict__ part_d,
               int *__restrict__ part_i, float *__restrict__ keys_out = nullptr, int64_t ldk = 0) {
    // LDS: two stages of A (queries) and B (db rows), 128×36 floats each; reused as the 128×128
    // distance tile in the epilogue (64 KiB ≤ 72 KiB).
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *As0 = smem;
    float *Bs0 = smem + GBM * GLD;
    float *As1 = smem + 2 * GBM * GLD;
    float *Bs1 = smem + 3 * GBM * GLD;
    float *Ct = smem;  // epilogue alias

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * GBM;
    const int64_t ntiles = ceil_div(N, GBN);
    const int64_t t0 = (int64_t)split * tiles_per_split;
    const int64_t t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int l31 = lane & 31, h = lane >> 5;

    WaveList<1, int> lists[WRITE ? 1 : 32];
#pragma unroll
    for (int r = 0; r < (WRITE ? 1 : 32); ++r) lists[r].init();

    const int nk = (d + GBK - 1) / GBK;
    float4 sa[4], sb[4];

    if (t0 < t1) {
        gemm_stage_load<VEC4>(Q, q0, nq, d, 0, sa);
        gemm_stage_load<VEC4>(X, t0 * GBN, N, d, 0, sb);
    }

    for (int64_t t = t0; t < t1; ++t) {
        const int64_t x0 = t * GBN;
        gemm_stage_store(As0, sa);
        gemm_stage_store(Bs0, sb);
        __syncthreads();

        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

        for (int kc = 0; kc < nk; ++kc) {
            const float *Ab = (kc & 1) ? As1 : As0;
            const float *Bb = (kc & 1) ? Bs1 : Bs0;
            if (kc + 1 < nk) {
                gemm_stage_load<VEC4>(Q, q0, nq, d, (kc + 1) * GBK, sa);
                gemm_stage_load<VEC4>(X, x0, N, d, (kc + 1) * GBK, sb);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                f32x4 a4[2], b4[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    a4[i] = *reinterpret_cast<const f32x4 *>(Ab + (64 * wr + 32 * i + l31) * GLD + 16 * h + 4 * u);
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    b4[j] = *reinterpret_cast<const f32x4 *>(Bb + (64 * wc + 32 * j + l31) * GLD + 16 * h + 4 * u);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[i][e], b4[j][e], acc[i][j], 0, 0, 0);
                }
            }
            if (kc + 1 < nk) {
                gemm_stage_store((kc & 1) ? As0 : As1, sa);
                gemm_stage_store((kc & 1) ? Bs0 : Bs1, sb);
            }
            __syncthreads();
        }

        // Prefetch the next tile's first K chunk while the epilogue runs.
        if (t + 1 < t1) {
            gemm_stage_load<VEC4>(Q, q0, nq, d, 0, sa);
            gemm_stage_load<VEC4>(X, (t + 1) * GBN, N, d, 0, sb);
        }

        if (WRITE) {  // keys straight from the accumulators to HBM
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int64_t q = q0 + 64 * wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const int64_t x = x0 + 64 * wc + 32 * j + l31;
                        if (q < nq && x < N) {
                            const float ip = acc[i][j][r];
                            float key;
                            if (metric == kL2) {
                                key = fmaf(-2.f, ip, qnorm[q] + xnorm[x]);
                                key = key < 0.f ? 0.f : key;
                            } else {
                                key = -ip;
                            }
                            keys_out[q * ldk + x] = key;
                        }
                    }
            continue;
        }
        // Epilogue 1: raw inner products → LDS tile Ct[128][128].
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 64 * wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int col = 64 * wc + 32 * j + l31;
                    Ct[row * GBN + col] = acc[i][j][r];
                }
        __syncthreads();

        // Epilogue 2: wave `wave` owns query rows [32*wave, 32*wave+32) of the tile.
        const int64_t xa = x0 + lane, xb = x0 + 64 + lane;
        const bool va = xa < N, vb = xb < N;
        float xna = 0.f, xnb = 0.f;
        if (metric == kL2) {
            xna = va ? xnorm[xa] : 0.f;
            xnb = vb ? xnorm[xb] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int row = 32 * wave + r;
            const int64_t q = q0 + row;
            if (q < nq) {  // wave-uniform
                const float ipa = Ct[row * GBN + lane];
                const float ipb = Ct[row * GBN + 64 + lane];
                float ka, kb;
                if (metric == kL2) {
                    const float qn = qnorm[q];
                    ka = fmaf(-2.f, ipa, qn + xna);
                    kb = fmaf(-2.f, ipb, qn + xnb);
                    ka = ka < 0.f ? 0.f : ka;
                    kb = kb < 0.f ? 0.f : kb;
                } else {
                    ka = -ipa;
                    kb = -ipb;
                }
                if (!va) ka = __builtin_inff();
                if (!vb) kb = __builtin_inff();
                lists[r].offer(ka, va ? (int)xa : 0x7fffffff, k - 1);
                lists[r].offer(kb, vb ? (int)xb : 0x7fffffff, k - 1);
            }
        }
        __syncthreads();
    }

    if (WRITE) return;
    // Store the per-(split, query) partial lists.
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const int64_t q = q0 + 32 * wave + r;
        if (q < nq) {
            const int64_t off = ((int64_t)split * nq + q) * k;
            lists[r].store(part_d + off, part_i + off, k);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// flat_gemm_topk2 — the fused path (k ≤ 64) with the selection state out of the register file.
//
// Same arithmetic as flat_gemm_topk (v_mfma_f32_32x32x2_f32, K chunks of 32, ‖q‖²+‖x‖²−2q·x clamped,
// or −q·x), different ownership: wave w owns the 32 query rows [32w, 32w+32) of the 128×128 tile
// across ALL 128 columns (acc[j], j = column block of 32), so a query's candidates never leave its
// wave.  Each query's sorted k-list lives in LDS; each lane holds the k-th key of the 16 queries its
// accumulator rows belong to (thr[r]: row (r&3) + 8(r>>2) + 4·half).  The epilogue compares the 64
// keys a lane holds with those thresholds straight from the accumulators (no LDS tile); a ballot per
// accumulator row sends the rare passing rows to the slow path, which loads that query's list into
// a WaveList, offers the 128 candidates (exact lexicographic admission) and writes it back.
//
// Registers ≈ 64 acc + 32 staging + 20 operands + 32 thr/‖q‖² + misc → ≤ 256 → 2 waves per SIMD; LDS
// = 64 KiB staging (XOR-swizzled, no padding) + 128·k·8 B lists → 2 blocks per CU for k ≤ 16.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int g2_swz(int row, int c4) { return c4 ^ ((row >> 1) & 7); }

__device__ __forceinline__ void g2_stage_store(float *__restrict__ lds, const float4 (&r)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int f = t + 256 * p;
        const int row = f >> 3, c4 = f & 7;
        *reinterpret_cast<float4 *>(lds + row * GBK + 4 * g2_swz(row, c4)) = r[p];
    }
}

size_t gemm2_smem_bytes(int k) { return (size_t)4 * GBM * GBK * sizeof(float) + (size_t)GBM * k * 8; }

// Epilogue of one 128×128 tile (wave = 32 query rows × 128 columns): keys straight from the
// accumulators, filtered by the per-row thresholds; rows with a passing key go through the WaveList.
template <bool L2M>
__device__ __forceinline__ void g2_epilogue(const f32x16 (&acc)[4], float (&thr)[16], const float (&qnv)[16],
                                            const float (&xnv)[4], int64_t x0, int64_t N, float *__restrict__ Ld,
                                            int *__restrict__ Li, int k, int wave, int lane) {
    const int l31 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float key[4];
        bool any = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float ip = acc[j][r];
            float kv;
            if (L2M) {
                kv = fmaf(-2.f, ip, qnv[r] + xnv[j]);
                kv = kv < 0.f ? 0.f : kv;
            } else {
                kv = -ip;
            }
            if (x0 + 32 * j + l31 >= N) kv = __builtin_inff();
            key[j] = kv;
            any |= kv <= thr[r];
        }
        const unsigned long long m = __ballot(any);
        if (m == 0ull) continue;
        // slow path (rare after the first tiles): each half of the wave is one query
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            if (((m >> (32 * hh)) & 0xffffffffull) == 0ull) continue;
            const int ql = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const int src = 32 * hh + l31;
            const float c0 = __shfl(key[0], src), c1 = __shfl(key[1], src);
            const float c2 = __shfl(key[2], src), c3 = __shfl(key[3], src);
            const float v0 = lane < 32 ? c0 : c1, v1 = lane < 32 ? c2 : c3;
            const int64_t col0 = x0 + (lane < 32 ? 0 : 32) + l31, col1 = col0 + 64;
            WaveList<1, int> L;
            L.d[0] = lane < k ? Ld[ql * k + lane] : __builtin_inff();
            L.id[0] = lane < k ? Li[ql * k + lane] : 0x7fffffff;
            L.offer(v0, col0 < N ? (int)col0 : 0x7fffffff, k - 1);
            L.offer(v1, col1 < N ? (int)col1 : 0x7fffffff, k - 1);
            if (lane < k) {
                Ld[ql * k + lane] = L.d[0];
                Li[ql * k + lane] = L.id[0];
            }
            const float nt = readlane_f(L.d[0], k - 1);
            if (h == hh) thr[r] = nt;
        }
    }
}

// per-(split, query) partial lists (each wave wrote only its own rows: no barrier needed)
// qmajor = 0: part[split][q][k] (merge_parts); qmajor = 1: part[q][split][k] (the exact form's rerank reads a
// query's lists contiguously)
__device__ __forceinline__ void g2_write_parts(const float *__restrict__ Ld, const int *__restrict__ Li, int64_t q0,
                                               int64_t nq, int k, int split, int wave, int lane,
                                               float *__restrict__ part_d, int *__restrict__ part_i, int nsplit = 0,
                                               int qmajor = 0) {
    for (int r = 0; r < 32; ++r) {
        const int ql = 32 * wave + r;
        const int64_t q = q0 + ql;
        if (q < nq && lane < k) {
            const int64_t off = (qmajor ? q * nsplit + split : (int64_t)split * nq + q) * k;
            part_d[off + lane] = Ld[ql * k + lane];
            part_i[off + lane] = Li[ql * k + lane];
        }
    }
}

template <bool VEC4, bool L2M>
__global__ void __launch_bounds__(256, 2)
flat_gemm_topk2(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq,
                const float *__restrict__ X, const float *__restrict__ xnorm, int64_t N, int d, int k, int nqt,
                int nsplit, int64_t tiles_per_split, float *__restrict__ part_d, int *__restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *As0 = smem;
    float *Bs0 = smem + GBM * GBK;
    float *As1 = smem + 2 * GBM * GBK;
    float *Bs1 = smem + 3 * GBM * GBK;
    float *Ld = smem + 4 * GBM * GBK;               // [128][k] keys
    int *Li = reinterpret_cast<int *>(Ld + GBM * k);  // [128][k] ids

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * GBM;
    const int64_t ntiles = ceil_div(N, GBN);
    const int64_t t0 = (int64_t)split * tiles_per_split;
    const int64_t t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int l31 = lane & 31, h = lane >> 5;
    const int arow = 32 * wave + l31;  // A operand row of this lane

    for (int e = tid; e < GBM * k; e += 256) {
        Ld[e] = __builtin_inff();
        Li[e] = 0x7fffffff;
    }
    // thresholds / ‖q‖² of the lane's accumulator rows; rows past nq never admit anything
    float thr[16], qnv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
        thr[r] = q < nq ? __builtin_inff() : -__builtin_inff();
        qnv[r] = (L2M && q < nq) ? qnorm[q] : 0.f;
    }
    __syncthreads();

    const int nk = (d + GBK - 1) / GBK;
    float4 sa[4], sb[4];
    if (t0 < t1) {
        gemm_stage_load<VEC4>(Q, q0, nq, d, 0, sa);
        gemm_stage_load<VEC4>(X, t0 * GBN, N, d, 0, sb);
    }

    for (int64_t t = t0; t < t1; ++t) {
        const int64_t x0 = t * GBN;
        g2_stage_store(As0, sa);
        g2_stage_store(Bs0, sb);
        float xnv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t x = x0 + 32 * j + l31;
            xnv[j] = (L2M && x < N) ? xnorm[x] : 0.f;
        }
        __syncthreads();

        f32x16 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

        for (int kc = 0; kc < nk; ++kc) {
            const float *Ab = (kc & 1) ? As1 : As0;
            const float *Bb = (kc & 1) ? Bs1 : Bs0;
            if (kc + 1 < nk) {
                gemm_stage_load<VEC4>(Q, q0, nq, d, (kc + 1) * GBK, sa);
                gemm_stage_load<VEC4>(X, x0, N, d, (kc + 1) * GBK, sb);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f32x4 a4 = *reinterpret_cast<const f32x4 *>(Ab + arow * GBK + 4 * g2_swz(arow, 4 * h + u));
                f32x4 b4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int brow = 32 * j + l31;
                    b4[j] = *reinterpret_cast<const f32x4 *>(Bb + brow * GBK + 4 * g2_swz(brow, 4 * h + u));
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[e], b4[j][e], acc[j], 0, 0, 0);
            }
            if (kc + 1 < nk) {
                g2_stage_store((kc & 1) ? As0 : As1, sa);
                g2_stage_store((kc & 1) ? Bs0 : Bs1, sb);
            }
            __syncthreads();
        }

        if (t + 1 < t1) {
            gemm_stage_load<VEC4>(Q, q0, nq, d, 0, sa);
            gemm_stage_load<VEC4>(X, (t + 1) * GBN, N, d, 0, sb);
        }

        g2_epilogue<L2M>(acc, thr, qnv, xnv, x0, N, Ld, Li, k, wave, lane);
    }
    g2_write_parts(Ld, Li, q0, nq, k, split, wave, lane, part_d, part_i);
}

// ---------------------------------------------------------------------------------------------
// flat_gemm_topk_bf — flat_gemm_topk2 with q·x on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16,
// 16× the fp32 matrix rate) over an NP-term round-to-nearest bf16 split of both operands: x = x₁ + x₂
// + x₃, each term the bf16 rounding of what the previous ones leave (exact fp32 subtractions).
//   NP = 3: x₁y₁ + x₁y₂ + x₂y₁ + x₁y₃ + x₃y₁ + x₂y₂ (the dropped products are ≤ 2⁻²⁶ relative):
//           fp32-level products, fp32 accumulation — the split of the IVF forms (ivf_mfma.hip).
//   NP = 2: x₁y₁ + x₁y₂ + x₂y₁, ≈ 2⁻¹⁶ relative per product (tuning / A-B only).
// Operands:
//   * queries: split once per batch (flat_split_queries) into qsplit [query][term][dpad] bf16 (dpad =
//     d rounded up to 32, zero-filled).  Each lane loads its A fragments (8 bf16 per MFMA) straight
//     from L2, one K chunk ahead: a 128-query tile's image is 128·dpad·2·NP B (590 KB at d = 768, 3
//     terms), re-read per database tile like flat_gemm_topk2's LDS-staged queries;
//   * database rows: the 128×32 fp32 chunk is loaded exactly as in flat_gemm_topk2 (coalesced float4
//     per lane, register staging one chunk ahead) and split while it is stored to LDS as
//     [term][16-B group c][row ^ 2c][8 bf16]: the XOR keeps the b64 stores (16-lane groups = 2 rows × 4
//     groups × 2 halves, banks (a/4) mod 32) and the b128 fragment reads (16-lane groups of 16 distinct
//     rows mod 16, banks (a/4) mod 64) conflict-free (MI355X_MICROARCH.md LDS table; row ^ 4c left the
//     stores 2-way conflicted: SQ_LDS_BANK_CONFLICT = 24 % of LDS cycles).
// MFMA s ∈ {0, 1} of a 32-dim chunk: lane half h holds dims 16s + 8h .. +7 of its A row and B column
// (group c = 2s + h).  Tile, grid, thresholds and the epilogue are flat_gemm_topk2's; LDS = 2 stages ×
// NP × 8 KiB + 128·k·8 B of lists → 2 blocks per CU for k ≤ 32 at NP = 3.
// ---------------------------------------------------------------------------------------------
typedef __bf16 fb_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 fb_bf16x2 __attribute__((ext_vector_type(2)));
typedef float fb_f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned fb_pack(float a, float b) {
    const fb_bf16x2 v = __builtin_convertvector((fb_f32x2){a, b}, fb_bf16x2);
    return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float fb_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float fb_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

// 4 fp32 → NP terms of 4 bf16 (two dwords each).  Scalar subtractions: v_pk_add_f32 beside MFMAs
// costs far more than its issue slot (MI355X_MICROARCH.md, price of one filler beside MFMAs).
template <int NP>
__device__ __forceinline__ void fb_split4(const float4 &v, uint2 (&o)[NP]) {
    float a = v.x, b = v.y, c = v.z, e = v.w;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const unsigned p0 = fb_pack(a, b), p1 = fb_pack(c, e);
        o[j] = make_uint2(p0, p1);
        if (j + 1 < NP) {
            a -= fb_lo(p0);
            b -= fb_hi(p0);
            c -= fb_lo(p1);
            e -= fb_hi(p1);
        }
    }
}

// LDS B stage: NP terms × 4 groups × 128 rows × 16 B
constexpr int FB_STAGE16 = 4 * GBN;  // 16-B units per term
__device__ __forceinline__ int fb_slot(int c, int row) { return c * GBN + (row ^ (c << 1)); }

// Row-chunk load for a T-thread block: the 128×32 fp32 chunk as 1024 float4, 1024/T per thread.
template <bool VEC4, int T>
__device__ __forceinline__ void fb_stage_load(const float *__restrict__ base, int64_t row0, int64_t nrows, int d,
                                              int k0, float4 (&r)[1024 / T]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 1024 / T; ++p) {
        const int f = t + T * p;
        const int row = f >> 3, c4 = f & 7;
        const int64_t grow = row0 + row;
        const int kk = k0 + 4 * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (grow < nrows) {
            const float *src = base + grow * (int64_t)d + kk;
            if (VEC4) {
                if (kk < d) v = *reinterpret_cast<const float4 *>(src);
            } else {
                if (kk + 0 < d) v.x = src[0];
                if (kk + 1 < d) v.y = src[1];
                if (kk + 2 < d) v.z = src[2];
                if (kk + 3 < d) v.w = src[3];
            }
        }
        r[p] = v;
    }
}

template <int NP, int T>
__device__ __forceinline__ void fb_stage_store(uint2 *__restrict__ lds, const float4 (&r)[1024 / T]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 1024 / T; ++p) {
        const int f = t + T * p;
        const int row = f >> 3, c4 = f & 7;
        uint2 o[NP];
        fb_split4<NP>(r[p], o);
        const int s = 2 * fb_slot(c4 >> 1, row) + (c4 & 1);
#pragma unroll
        for (int j = 0; j < NP; ++j) lds[j * 2 * FB_STAGE16 + s] = o[j];
    }
}

// term pairs (A term, B term) of the products, smallest first
template <int NP>
struct FbProducts;
template <>
struct FbProducts<3> {
    static constexpr int n = 6;
    __device__ static constexpr int a(int i) { return i == 0 ? 2 : i == 1 ? 0 : i == 2 ? 1 : i == 3 ? 0 : i == 4 ? 1 : 0; }
    __device__ static constexpr int b(int i) { return i == 0 ? 0 : i == 1 ? 2 : i == 2 ? 1 : i == 3 ? 1 : i == 4 ? 0 : 0; }
};
template <>
struct FbProducts<2> {
    static constexpr int n = 3;
    __device__ static constexpr int a(int i) { return i == 0 ? 1 : 0; }
    __device__ static constexpr int b(int i) { return i == 1 ? 1 : 0; }
};

size_t gemm_bf_smem_bytes(int np, int k, int w) { return (size_t)2 * np * FB_STAGE16 * 16 + (size_t)32 * w * k * 8; }
// the largest list length k (≤ 64) whose LDS lists fit either block shape
int flat_gemm_topk_bf_kmax(int np) {
    int k = 64;
    while (k > 1 && gemm_bf_smem_bytes(np, k, 8) > 160 * 1024) --k;
    return k;
}

template <bool VEC4, bool L2M, int NP, int W>
__global__ void __launch_bounds__(64 * W, 8 / W)
flat_gemm_topk_bf(const uint4 *__restrict__ qsplit, int dpad, const float *__restrict__ qnorm, int64_t nq,
                  const float *__restrict__ X, const float *__restrict__ xnorm, int64_t N, int d, int k, int nqt,
                  int nsplit, int64_t tiles_per_split, float *__restrict__ part_d, int *__restrict__ part_i,
                  int qmajor) {
    constexpr int TH = 64 * W, QM = 32 * W;  // threads; query rows per block (32 per wave)
    extern __shared__ __attribute__((aligned(16))) uint4 smem_bf[];
    uint4 *Bs0 = smem_bf;
    uint4 *Bs1 = smem_bf + NP * FB_STAGE16;
    float *Ld = reinterpret_cast<float *>(smem_bf + 2 * NP * FB_STAGE16);  // [QM][k] keys
    int *Li = reinterpret_cast<int *>(Ld + QM * k);                         // [QM][k] ids

    const int nblocks = nqt * nsplit;
    const int lb = xcd_remap(blockIdx.x, nblocks);
    const int qt = lb % nqt;
    const int split = lb / nqt;
    const int64_t q0 = (int64_t)qt * QM;
    const int64_t ntiles = ceil_div(N, GBN);
    const int64_t t0 = (int64_t)split * tiles_per_split;
    const int64_t t1 = t0 + tiles_per_split < ntiles ? t0 + tiles_per_split : ntiles;

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int l31 = lane & 31, h = lane >> 5;

    for (int e = tid; e < QM * k; e += TH) {
        Ld[e] = __builtin_inff();
        Li[e] = 0x7fffffff;
    }
    float thr[16], qnv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
        thr[r] = q < nq ? __builtin_inff() : -__builtin_inff();
        qnv[r] = (L2M && q < nq) ? qnorm[q] : 0.f;
    }
    // this lane's A row (rows past nq re-read the last query; their thresholds admit nothing)
    int64_t qa = q0 + 32 * wave + l31;
    qa = qa < nq ? qa : nq - 1;
    const int dq = dpad >> 3;  // 16-B units per query term
    const uint4 *qrow = qsplit + qa * NP * dq + h;
    __syncthreads();

    const int nk = dpad / GBK;
    float4 sb[1024 / TH];
    uint4 af[NP][2], an[NP][2];
    if (t0 < t1) {
        fb_stage_load<VEC4, TH>(X, t0 * GBN, N, d, 0, sb);
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) af[j][s] = qrow[j * dq + 2 * s];
    }

    for (int64_t t = t0; t < t1; ++t) {
        const int64_t x0 = t * GBN;
        fb_stage_store<NP, TH>(reinterpret_cast<uint2 *>(Bs0), sb);
        float xnv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t x = x0 + 32 * j + l31;
            xnv[j] = (L2M && x < N) ? xnorm[x] : 0.f;
        }
        __syncthreads();

        f32x16 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

        for (int kc = 0; kc < nk; ++kc) {
            const uint4 *Bb = (kc & 1) ? Bs1 : Bs0;
            if (kc + 1 < nk) fb_stage_load<VEC4, TH>(X, x0, N, d, (kc + 1) * GBK, sb);
            const int kn = kc + 1 < nk ? kc + 1 : 0;  // the next tile starts over at chunk 0
#pragma unroll
            for (int j = 0; j < NP; ++j)
#pragma unroll
                for (int s = 0; s < 2; ++s) an[j][s] = qrow[j * dq + 4 * kn + 2 * s];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int c = 2 * s + h;
#pragma unroll
                for (int jb = 0; jb < 4; ++jb) {
                    uint4 bt[NP];
#pragma unroll
                    for (int j = 0; j < NP; ++j) bt[j] = Bb[j * FB_STAGE16 + fb_slot(c, 32 * jb + l31)];
#pragma unroll
                    for (int pr = 0; pr < FbProducts<NP>::n; ++pr)
                        acc[jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                            __builtin_bit_cast(fb_bf16x8, af[FbProducts<NP>::a(pr)][s]),
                            __builtin_bit_cast(fb_bf16x8, bt[FbProducts<NP>::b(pr)]), acc[jb], 0, 0, 0);
                }
            }
            if (kc + 1 < nk) fb_stage_store<NP, TH>(reinterpret_cast<uint2 *>((kc & 1) ? Bs0 : Bs1), sb);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < NP; ++j)
#pragma unroll
                for (int s = 0; s < 2; ++s) af[j][s] = an[j][s];
        }

        if (t + 1 < t1) fb_stage_load<VEC4, TH>(X, (t + 1) * GBN, N, d, 0, sb);
        g2_epilogue<L2M>(acc, thr, qnv, xnv, x0, N, Ld, Li, k, wave, lane);
    }
    g2_write_parts(Ld, Li, q0, nq, k, split, wave, lane, part_d, part_i, nsplit, qmajor);
}

// The batch's queries split once into NP bf16 terms: qsplit [query][term][dpad] (dims in order, zero
// past d).  One thread per 4 dims.
template <int NP>
__global__ void __launch_bounds__(256) flat_split_queries(const float *__restrict__ Q, int64_t nq, int d, int dpad,
                                                          uint2 *__restrict__ qs) {
    const int ng = dpad >> 2;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nq * ng) return;
    const int64_t q = i / ng;
    const int g = (int)(i - q * ng), dim = 4 * g;
    const float *src = Q + q * (int64_t)d + dim;
    float4 v;
    v.x = dim + 0 < d ? src[0] : 0.f;
    v.y = dim + 1 < d ? src[1] : 0.f;
    v.z = dim + 2 < d ? src[2] : 0.f;
    v.w = dim + 3 < d ? src[3] : 0.f;
    uint2 o[NP];
    fb_split4<NP>(v, o);
#pragma unroll
    for (int j = 0; j < NP; ++j) qs[(q * NP + j) * ng + g] = o[j];
}

// ---------------------------------------------------------------------------------------------
// flat_scan_topk — direct-form streaming scan for small query batches (FAISS nq < 20 path,
// fvec_L2sqr / fvec_inner_product).  Queries live in LDS; each wave walks a contiguous range of
// database rows, R rows at a time (R float4 row loads in flight per lane), reduces Σ(q−x)² (or
// q·x) across the wave and keeps one top-k list per query.  HBM-bound: every X byte read once.
// Partial lists go to part[(wave_global * nq + q) * k].
// ---------------------------------------------------------------------------------------------
constexpr int SCAN_R = 4;

template <int NQ, bool VEC4, bool WRITE = false>
__global__ void __launch_bounds__(256)
flat_scan_topk(const float *__restrict__ Q, const float *__restrict__ X, int64_t N, int d, int metric, int k,
               int64_t rows_per_wave, float *__restrict__ part_d, int *__restrict__ part_i,
               float *__restrict__ keys_out = nullptr, int64_t ldk = 0) {
    extern __shared__ __attribute__((aligned(16))) float qs[];  // NQ × dpad
    const int dpad = (d + 3) & ~3;
    for (int i = threadIdx.x; i < NQ * dpad; i += 256) {
        const int qi = i / dpad, j = i - qi * dpad;
        qs[i] = j < d ? Q[(int64_t)qi * d + j] : 0.f;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t r0 = gw * rows_per_wave;
    int64_t r1 = r0 + rows_per_wave;
    if (r1 > N) r1 = N;

    WaveList<1, int> lists[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) lists[qi].init();

    // Per-lane candidate slots: after each group of 64 rows, lane j holds row (base + j).
    float cand[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) cand[qi] = __builtin_inff();

    const int nd4 = dpad >> 2;
    for (int64_t base = r0; base < r1; base += 64) {
        const int64_t gend = (base + 64 < r1) ? base + 64 : r1;
        for (int64_t rr = base; rr < gend; rr += SCAN_R) {
            float acc[SCAN_R][NQ];
#pragma unroll
            for (int r = 0; r < SCAN_R; ++r)
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) acc[r][qi] = 0.f;
            for (int j4 = lane; j4 < nd4; j4 += 64) {
                float4 xv[SCAN_R];
#pragma unroll
                for (int r = 0; r < SCAN_R; ++r) {
                    const int64_t row = rr + r;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (row < gend) {
                        const float *src = X + row * (int64_t)d + 4 * j4;
                        if (VEC4) v = *reinterpret_cast<const float4 *>(src);
                        else {
                            const int j = 4 * j4;
                            if (j + 0 < d) v.x = src[0];
                            if (j + 1 < d) v.y = src[1];
                            if (j + 2 < d) v.z = src[2];
                            if (j + 3 < d) v.w = src[3];
                        }
                    }
                    xv[r] = v;
                }
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
                    const float4 qv = *reinterpret_cast<const float4 *>(qs + qi * dpad + 4 * j4);
#pragma unroll
                    for (int r = 0; r < SCAN_R; ++r) {
                        if (metric == kL2) {
                            float t;
                            t = qv.x - xv[r].x; acc[r][qi] = fmaf(t, t, acc[r][qi]);
                            t = qv.y - xv[r].y; acc[r][qi] = fmaf(t, t, acc[r][qi]);
                            t = qv.z - xv[r].z; acc[r][qi] = fmaf(t, t, acc[r][qi]);
                            t = qv.w - xv[r].w; acc[r][qi] = fmaf(t, t, acc[r][qi]);
                        } else {
                            acc[r][qi] = fmaf(qv.x, xv[r].x, acc[r][qi]);
                            acc[r][qi] = fmaf(qv.y, xv[r].y, acc[r][qi]);
                            acc[r][qi] = fmaf(qv.z, xv[r].z, acc[r][qi]);
                            acc[r][qi] = fmaf(qv.w, xv[r].w, acc[r][qi]);
                        }
                    }
                }
            }
            // Wave reductions; row rr+r lands in lane (rr + r - base).
#pragma unroll
            for (int r = 0; r < SCAN_R; ++r) {
                const int slot = (int)(rr + r - base);
#pragma unroll
                for (int qi = 0; qi < NQ; ++qi) {
                    float s = acc[r][qi];
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
                    if (metric != kL2) s = -s;
                    if (lane == slot) cand[qi] = s;
                }
            }
        }
        // Offer the (up to) 64 candidates of this group (or write them out).
        const int64_t myrow = base + lane;
        const bool valid = myrow < gend;
#pragma unroll
        for (int qi = 0; qi < NQ; ++qi) {
            if (WRITE) {
                if (valid) keys_out[qi * ldk + myrow] = cand[qi];
            } else {
                lists[qi].offer(valid ? cand[qi] : __builtin_inff(), valid ? (int)myrow : 0x7fffffff, k - 1);
            }
        }
    }
    if (WRITE) return;
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) {
        const int64_t off = (gw * NQ + qi) * (int64_t)k;
        lists[qi].store(part_d + off, part_i + off, k);
    }
}

// ---------------------------------------------------------------------------------------------
// merge_parts_topk — per query, the k best of nparts partial lists laid out [part][nq][k].
// Keys are "smaller is better" (L2 distance or −IP).  One wave per query; S = ceil(k/64).
//   in_local:  ids are int32 row numbers local to this index (label = label_offset + id)
//   out_sign:  +1 → D = key; −1 → D = −key (IP: back to raw dot products)
// Pads ((+inf, pad) or label < 0) become (±inf, −1).
// ---------------------------------------------------------------------------------------------
template <int S, typename InId>
__global__ void __launch_bounds__(256)
merge_parts_topk(const float *__restrict__ pd, const InId *__restrict__ pi, int nparts, int64_t nq, int k,
                 int kout, int64_t label_offset, float in_sign, float out_sign, float *__restrict__ D,
                 int64_t *__restrict__ I, int64_t pstride_d, int64_t pstride_i) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<S, long long> L;
    L.init();
    const int64_t total = (int64_t)nparts * k;
    constexpr int MU = 4;  // 64-candidate chunks loaded ahead of their offers
    for (int64_t c0 = 0; c0 < total; c0 += 64 * MU) {
        float key[MU];
        long long lab[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t c = c0 + 64 * u + lane;
            key[u] = __builtin_inff();
            lab[u] = IdTraits<long long>::pad();
            if (c < total) {
                const int64_t p = c / k, i = c - p * k;
                const InId raw = pi[p * pstride_i + q * k + i];
                const float v = pd[p * pstride_d + q * k + i] * in_sign;
                // int32 partials pad with 0x7fffffff; int64 (global label) partials only with negatives, so a
                // real label 2^31 - 1 (arbitrary IVF ids, > 2^31 rows) is kept
                bool pad_in = raw < 0;
                if constexpr (sizeof(InId) == 4) pad_in = pad_in || raw == (InId)0x7fffffff;
                if (!pad_in && !(v == __builtin_inff())) {
                    key[u] = v;
                    lab[u] = (long long)raw + label_offset;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < MU; ++u) L.offer(key[u], lab[u], kout - 1);
    }
    const float pad_d = out_sign > 0.f ? __builtin_inff() : -__builtin_inff();
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int e = s * 64 + lane;
        if (e < kout) {
            const bool pad = L.id[s] == IdTraits<long long>::pad();
            D[q * kout + e] = pad ? pad_d : L.d[s] * out_sign;
            I[q * kout + e] = pad ? -1 : (int64_t)L.id[s];
        }
    }
}

// merge_parts_stage1 — the first level of a two-level merge (many parts, few queries: the direct scan's
// 8192 per-wave lists at nq = 1 kept ONE wave busy for ~1 ms).  Wave (g, q) merges parts
// [g·ppg, (g+1)·ppg) of query q into one (key, label) list of kout written to [g][q][kout] (labels global,
// pads (+inf, −1)); merge_parts_topk then merges the G group lists.  Lexicographic top-k is associative,
// so the result equals the one-level merge.
template <typename InId>
__global__ void __launch_bounds__(256)
merge_parts_stage1(const float *__restrict__ pd, const InId *__restrict__ pi, int nparts, int64_t nq, int k, int kout,
                   int64_t label_offset, float in_sign, int ppg, int ngroups, float *__restrict__ md,
                   long long *__restrict__ mi) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= (int64_t)ngroups * nq) return;
    const int64_t q = w % nq, g = w / nq;
    const int lane = threadIdx.x & 63;
    const int p0 = (int)g * ppg, p1 = p0 + ppg < nparts ? p0 + ppg : nparts;
    const int64_t total = (int64_t)(p1 - p0) * k;
    WaveList<1, long long> L;
    L.init();
    constexpr int MU = 4;
    for (int64_t c0 = 0; c0 < total; c0 += 64 * MU) {
        float key[MU];
        long long lab[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t c = c0 + 64 * u + lane;
            key[u] = __builtin_inff();
            lab[u] = IdTraits<long long>::pad();
            if (c < total) {
                const int64_t p = p0 + c / k, i = c % k;
                const InId raw = pi[(p * nq + q) * k + i];
                const float v = pd[(p * nq + q) * k + i] * in_sign;
                bool pad_in = raw < 0;
                if constexpr (sizeof(InId) == 4) pad_in = pad_in || raw == (InId)0x7fffffff;
                if (!pad_in && !(v == __builtin_inff())) {
                    key[u] = v;
                    lab[u] = (long long)raw + label_offset;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < MU; ++u) L.offer(key[u], lab[u], kout - 1);
    }
    if (lane < kout) {
        const bool pad = L.id[0] == IdTraits<long long>::pad();
        md[w * kout + lane] = pad ? __builtin_inff() : L.d[0];
        mi[w * kout + lane] = pad ? -1 : L.id[0];
    }
}

// merge_groups_block — the second level: one 4-wave block per query, each wave merging a quarter of the
// ngroups group lists ([g][q][kout], global labels, −1 pads), wave 0 merging the four wave lists through LDS.
__global__ void __launch_bounds__(256)
merge_groups_block(const float *__restrict__ md, const long long *__restrict__ mi, int ngroups, int64_t nq, int kout,
                   float out_sign, float *__restrict__ D, int64_t *__restrict__ I) {
    __shared__ float sd[4 * 64];
    __shared__ long long si[4 * 64];
    const int64_t q = blockIdx.x;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g0 = (int)((int64_t)ngroups * wv / 4), g1 = (int)((int64_t)ngroups * (wv + 1) / 4);
    const int64_t total = (int64_t)(g1 - g0) * kout;
    WaveList<1, long long> L;
    L.init();
    constexpr int MU = 4;
    for (int64_t c0 = 0; c0 < total; c0 += 64 * MU) {
        float key[MU];
        long long lab[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t c = c0 + 64 * u + lane;
            key[u] = __builtin_inff();
            lab[u] = IdTraits<long long>::pad();
            if (c < total) {
                const int64_t g = g0 + c / kout, i = c % kout;
                const long long raw = mi[(g * nq + q) * kout + i];
                const float v = md[(g * nq + q) * kout + i];
                if (raw >= 0 && !(v == __builtin_inff())) {
                    key[u] = v;
                    lab[u] = raw;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < MU; ++u) L.offer(key[u], lab[u], kout - 1);
    }
    sd[wv * 64 + lane] = L.d[0];
    si[wv * 64 + lane] = L.id[0];
    __syncthreads();
    if (wv != 0) return;
    L.init();
#pragma unroll
    for (int w = 0; w < 4; ++w) L.offer(sd[w * 64 + lane], si[w * 64 + lane], kout - 1);
    if (lane < kout) {
        const bool pad = L.id[0] == IdTraits<long long>::pad();
        D[q * kout + lane] = pad ? (out_sign > 0.f ? __builtin_inff() : -__builtin_inff()) : L.d[0] * out_sign;
        I[q * kout + lane] = pad ? -1 : (int64_t)L.id[0];
    }
}

// ---------------------------------------------------------------------------------------------
// rows_topk — k > 64 path: per (query row, column segment) one wave with an S-slot list over
// keys[q * ldk + c], c in the segment; ids = id0 + c.  Partials go to [seg][q][k].
// ---------------------------------------------------------------------------------------------
template <int S>
__global__ void __launch_bounds__(256)
rows_topk(const float *__restrict__ keys, int64_t ldk, int64_t ncols, int64_t nq, int64_t seg_len, int nseg, int k,
          int id0, float *__restrict__ part_d, int *__restrict__ part_i) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nq * nseg) return;
    const int64_t q = w % nq, sg = w / nq;
    const int lane = threadIdx.x & 63;
    WaveList<S, int> L;
    L.init();
    const int64_t c0 = sg * seg_len;
    const int64_t c1 = c0 + seg_len < ncols ? c0 + seg_len : ncols;
    for (int64_t c = c0; c < c1; c += 64) {
        const int64_t cc = c + lane;
        const bool v = cc < c1;
        L.offer(v ? keys[q * ldk + cc] : __builtin_inff(), v ? (int)(id0 + cc) : 0x7fffffff, k - 1);
    }
    const int64_t off = (sg * nq + q) * (int64_t)k;
    L.store(part_d + off, part_i + off, k);
}

// rows_select_out — a whole key row per wave straight to the output (one-chunk tables: the IVF coarse
// quantizer's nq × nlist keys).  The lexicographic (key, column) top-k of the row, written as
// merge_parts_topk writes it (D = key·out_sign, I = label_offset + column; +inf keys and empty slots
// become (±inf, −1)) — identical to rows_topk over segments + merge_parts_topk, in one launch with
// every key load of the row in flight at once.
template <int S>
__global__ void __launch_bounds__(256)
rows_select_out(const float *__restrict__ keys, int64_t ldk, int64_t ncols, int64_t nq, int k, int kout,
                int64_t label_offset, float out_sign, float *__restrict__ D, int64_t *__restrict__ I) {
    constexpr int U = 8;  // 64-column chunks loaded ahead of their offers
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    const float *row = keys + q * ldk;
    WaveList<S, int> L;
    L.init();
    for (int64_t c0 = 0; c0 < ncols; c0 += 64 * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c = c0 + 64 * u + lane;
            v[u] = c < ncols ? row[c] : __builtin_inff();
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t c = c0 + 64 * u + lane;
            L.offer(v[u], c < ncols ? (int)c : 0x7fffffff, k - 1);
        }
    }
    const float pad_d = out_sign > 0.f ? __builtin_inff() : -__builtin_inff();
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int e = s * 64 + lane;
        if (e < kout) {
            const bool pad = e >= k || L.id[s] == 0x7fffffff || L.d[s] == __builtin_inff();
            D[q * kout + e] = pad ? pad_d : L.d[s] * out_sign;
            I[q * kout + e] = pad ? -1 : (int64_t)L.id[s] + label_offset;
        }
    }
}

// rows_select_small — the same output for rows of ≤ 64·J columns and k ≤ 64, without serial inserts:
// the row sits in registers (J keys per lane, column 64j + lane) as order-preserving u32 (±0 merged, NaN
// never selected — as lex_less never admits it); the k-th smallest value T comes from a 32-step bitwise
// search (each step: J ballots + popcounts), the keys < T and then the first (by column) keys == T are
// compacted through LDS, and one bitonic wave sort orders them by (key, column).  ≈ 1.5K instructions
// per row against the ≈ 20 latency-bound serial inserts per row of the list path (1024 × 1024, k 32:
// 41 µs with the list path).
template <int J>
__global__ void __launch_bounds__(256)
rows_select_small(const float *__restrict__ keys, int64_t ldk, int ncols, int64_t nq, int k, int kout,
                  int64_t label_offset, float out_sign, float *__restrict__ D, int64_t *__restrict__ I,
                  const int *__restrict__ list_len, int nlist, int chunk_rows, int *__restrict__ ccnt,
                  int *__restrict__ slot_off, int *__restrict__ qtot) {
    __shared__ float sk[4][64];
    __shared__ int sc[4][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + wv;
    const bool live = q < nq;  // wave-uniform; every wave reaches the barrier
    const float *row = keys + (live ? q : 0) * ldk;
    float v[J];
    unsigned u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = 64 * j + lane;
        v[j] = live && c < ncols ? row[c] : __builtin_nanf("");
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const float f = v[j] == 0.f ? 0.f : v[j];
        const unsigned b = __float_as_uint(f);
        u[j] = v[j] == v[j] ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
    }
    unsigned T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = T | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) cnt += __popcll(__ballot(u[j] < cand));
        if (cnt < k) T = cand;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    int base = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool s = u[j] < T;
        const unsigned long long m = __ballot(s);
        if (s) {
            const int pos = base + __popcll(m & lt);
            sk[wv][pos] = v[j];
            sc[wv][pos] = 64 * j + lane;
        }
        base += __popcll(m);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool s = u[j] == T && u[j] != 0xffffffffu;
        const unsigned long long m = __ballot(s);
        if (s) {
            const int pos = base + __popcll(m & lt);
            if (pos < k) {
                sk[wv][pos] = v[j];
                sc[wv][pos] = 64 * j + lane;
            }
        }
        base += __popcll(m);
    }
    const int nsel = base < k ? base : k;
    __syncthreads();
    float kk = lane < nsel ? sk[wv][lane] : __builtin_inff();
    int cc = lane < nsel ? sc[wv][lane] : 0x7fffffff;
    wave_rank_sort(kk, cc, nsel);
    const bool pad = lane >= nsel || kk == __builtin_inff();
    if (live && lane < kout) {
        D[q * kout + lane] = pad ? (out_sign > 0.f ? __builtin_inff() : -__builtin_inff()) : kk * out_sign;
        I[q * kout + lane] = pad ? -1 : (int64_t)cc + label_offset;
    }
    if (ccnt && live) {  // the IVF plan's per-query step (ivf_count_q) on the probes just selected (kout ≤ 64)
        const int64_t l = lane < kout && !pad ? (int64_t)cc + label_offset : -1;
        const int len = l >= 0 && l < nlist ? list_len[l] : 0;
        if (len > 0) atomicAdd(ccnt + (int64_t)(q % kPlanCopies) * nlist + l, 1);
        const int v = len > 0 ? (len + chunk_rows - 1) / chunk_rows : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        if (lane < kout) slot_off[q * kout + lane] = x - v;
        if (lane == 63) qtot[q] = x;
    }
}

// rows_select_narrow — rows_select_small's output (and the IVF plan's count step) for rows of 257..64·J keys, one wave
// per row, narrowed as flat_keys_kth: T_hi = the k-th smallest of the 64 lanes' minima (k keys lie at or below it, so
// the k-th smallest key does too), the keys ≤ T_hi compacted into LDS in column order (≈ k + a few for i.i.d. rows),
// then the exact k-th T over that list by the one-register bitwise search and the take (keys < T, then the first keys
// == T by column) — the same k (key, column) pairs as the search over the whole row, in 2 × 32 one-ballot steps
// instead of 32 × J.  A list longer than 64 (a row with more than 64 keys at or below T_hi) takes the whole-row search.
// r05: the coarse select of the IVF headline 12.9 → see DESIGN §5; the extension's nq = 1 call 9.7 µs (one
// block's 32 barrier-separated steps) → one wave.
template <int J>
__global__ void __launch_bounds__(256)
rows_select_narrow(const float *__restrict__ keys, int64_t ldk, int ncols, int64_t nq, int k, int kout,
                   int64_t label_offset, float out_sign, float *__restrict__ D, int64_t *__restrict__ I,
                   const int *__restrict__ list_len, int nlist, int chunk_rows, int *__restrict__ ccnt,
                   int *__restrict__ slot_off, int *__restrict__ qtot) {
    __shared__ float sk[4][64];
    __shared__ int sc[4][64];
    __shared__ float tk[4][64];
    __shared__ int tc[4][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + wv;
    if (q >= nq) return;  // (no block barrier below: each wave's LDS rows are its own)
    const float *row = keys + q * ldk;
    float v[J];
    unsigned u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = 64 * j + lane;
        v[j] = c < ncols ? row[c] : __builtin_nanf("");
    }
    unsigned mn = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const float f = v[j] == 0.f ? 0.f : v[j];
        const unsigned b = __float_as_uint(f);
        u[j] = v[j] == v[j] ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
        mn = min(mn, u[j]);
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    // T_hi: the k-th smallest lane minimum (as rows_select_small's search: the largest T with #{< T} < k)
    unsigned th = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = th | (1u << bit);
        if ((int)__popcll(__ballot(mn < cand)) < k) th = cand;
    }
    // the keys ≤ T_hi in column order
    int c = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool a = u[j] <= th && u[j] != 0xffffffffu;
        const unsigned long long ma = __ballot(a);
        const int p = c + (int)__popcll(ma & lt);
        if (a && p < 64) { tk[wv][p] = v[j]; tc[wv][p] = 64 * j + lane; }
        c += (int)__popcll(ma);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    unsigned T = 0;
    if (c <= 64) {
        const float f0 = lane < c ? tk[wv][lane] : 0.f;
        const float f = f0 == 0.f ? 0.f : f0;
        const unsigned b = __float_as_uint(f);
        const unsigned ul = lane < c ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
        for (int bit = 31; bit >= 0; --bit) {
            const unsigned cand = T | (1u << bit);
            if ((int)__popcll(__ballot(ul < cand)) < k) T = cand;
        }
    } else {  // the whole row
        for (int bit = 31; bit >= 0; --bit) {
            const unsigned cand = T | (1u << bit);
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < J; ++j) cnt += __popcll(__ballot(u[j] < cand));
            if (cnt < k) T = cand;
        }
    }
    // the take, from the row's registers (column order): keys < T, then the first keys == T
    int base = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool s = u[j] < T;
        const unsigned long long m = __ballot(s);
        if (s) {
            const int pos = base + __popcll(m & lt);
            sk[wv][pos] = v[j];
            sc[wv][pos] = 64 * j + lane;
        }
        base += __popcll(m);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool s = u[j] == T && u[j] != 0xffffffffu;
        const unsigned long long m = __ballot(s);
        if (s) {
            const int pos = base + __popcll(m & lt);
            if (pos < k) {
                sk[wv][pos] = v[j];
                sc[wv][pos] = 64 * j + lane;
            }
        }
        base += __popcll(m);
    }
    const int nsel = base < k ? base : k;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float kk = lane < nsel ? sk[wv][lane] : __builtin_inff();
    int cc = lane < nsel ? sc[wv][lane] : 0x7fffffff;
    wave_rank_sort(kk, cc, nsel);
    const bool pad = lane >= nsel || kk == __builtin_inff();
    if (lane < kout) {
        D[q * kout + lane] = pad ? (out_sign > 0.f ? __builtin_inff() : -__builtin_inff()) : kk * out_sign;
        I[q * kout + lane] = pad ? -1 : (int64_t)cc + label_offset;
    }
    if (ccnt) {  // the IVF plan's per-query step (ivf_count_q) on the probes just selected (kout ≤ 64)
        const int64_t l = lane < kout && !pad ? (int64_t)cc + label_offset : -1;
        const int len = l >= 0 && l < nlist ? list_len[l] : 0;
        if (len > 0) atomicAdd(ccnt + (int64_t)(q % kPlanCopies) * nlist + l, 1);
        const int vv = len > 0 ? (len + chunk_rows - 1) / chunk_rows : 0;
        int x = vv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        if (lane < kout) slot_off[q * kout + lane] = x - vv;
        if (lane == 63) qtot[q] = x;
    }
}

// rows_select_block — rows of 257..1024 keys: rows_select_small's select with the row spread over a
// block of 4 waves (column c = 256·wave + 64·j + lane, J = 4 registers per lane); each search step sums
// the waves' ballot counts through LDS (one barrier), the compaction runs in (wave, j, lane) = column
// order, and wave 0 sorts and writes the output (and the IVF plan's count step).  A quarter of the
// per-wave ballot chain of the one-wave version (16 µs for 1024 × 1024 keys).  Measured and rejected (r04): a
// one-barrier variant (each wave selects its 256 columns' k best, wave 0 merges): 13.5 µs, the same — the
// barriers are not the critical path.
__global__ void __launch_bounds__(256)
rows_select_block(const float *__restrict__ keys, int64_t ldk, int ncols, int64_t nq, int k, int kout,
                  int64_t label_offset, float out_sign, float *__restrict__ D, int64_t *__restrict__ I,
                  const int *__restrict__ list_len, int nlist, int chunk_rows, int *__restrict__ ccnt,
                  int *__restrict__ slot_off, int *__restrict__ qtot) {
    constexpr int J = 4, WV = 4;
    __shared__ float sk[64];
    __shared__ int sc[64];
    __shared__ int scnt[2][WV];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = blockIdx.x;
    const float *row = keys + q * ldk;
    float v[J];
    unsigned u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = 256 * wv + 64 * j + lane;
        v[j] = c < ncols ? row[c] : __builtin_nanf("");
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const float f = v[j] == 0.f ? 0.f : v[j];
        const unsigned b = __float_as_uint(f);
        u[j] = v[j] == v[j] ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
    }
    unsigned T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = T | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) cnt += __popcll(__ballot(u[j] < cand));
        const int par = bit & 1;
        if (lane == 0) scnt[par][wv] = cnt;
        __syncthreads();
        const int tot = scnt[par][0] + scnt[par][1] + scnt[par][2] + scnt[par][3];
        if (tot < k) T = cand;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    int nlt = 0, neq = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        nlt += __popcll(__ballot(u[j] < T));
        neq += __popcll(__ballot(u[j] == T && u[j] != 0xffffffffu));
    }
    __syncthreads();  // every wave has read the last search step's counts
    if (lane == 0) { scnt[0][wv] = nlt; scnt[1][wv] = neq; }
    __syncthreads();
    int olt = 0, oeq = 0, tlt = 0, teq = 0;
#pragma unroll
    for (int w = 0; w < WV; ++w) {
        olt += w < wv ? scnt[0][w] : 0;
        oeq += w < wv ? scnt[1][w] : 0;
        tlt += scnt[0][w];
        teq += scnt[1][w];
    }
    int plt = olt, peq = tlt + oeq;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool a = u[j] < T, b = u[j] == T && u[j] != 0xffffffffu;
        const unsigned long long ma = __ballot(a), mb = __ballot(b);
        const int c = 256 * wv + 64 * j + lane;
        if (a) { const int p = plt + __popcll(ma & lt); sk[p] = v[j]; sc[p] = c; }
        if (b) { const int p = peq + __popcll(mb & lt); if (p < k) { sk[p] = v[j]; sc[p] = c; } }
        plt += __popcll(ma);
        peq += __popcll(mb);
    }
    const int nsel = tlt + teq < k ? tlt + teq : k;
    __syncthreads();
    if (wv != 0) return;
    float kk = lane < nsel ? sk[lane] : __builtin_inff();
    int cc = lane < nsel ? sc[lane] : 0x7fffffff;
    wave_rank_sort(kk, cc, nsel);
    const bool pad = lane >= nsel || kk == __builtin_inff();
    if (lane < kout) {
        D[q * kout + lane] = pad ? (out_sign > 0.f ? __builtin_inff() : -__builtin_inff()) : kk * out_sign;
        I[q * kout + lane] = pad ? -1 : (int64_t)cc + label_offset;
    }
    if (ccnt) {  // the IVF plan's per-query step (ivf_count_q) on the probes just selected (kout ≤ 64)
        const int64_t l = lane < kout && !pad ? (int64_t)cc + label_offset : -1;
        const int len = l >= 0 && l < nlist ? list_len[l] : 0;
        if (len > 0) atomicAdd(ccnt + (int64_t)(q % kPlanCopies) * nlist + l, 1);
        const int vv = len > 0 ? (len + chunk_rows - 1) / chunk_rows : 0;
        int x = vv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        if (lane < kout) slot_off[q * kout + lane] = x - vv;
        if (lane == 63) qtot[q] = x;
    }
}


// Raw merge: nparts partial [part][nq][k] (keys, int ids) → one [nq][k] partial (keys, int ids).
template <int S>
__global__ void __launch_bounds__(256)
merge_parts_raw(const float *__restrict__ pd, const int *__restrict__ pi, int nparts, int64_t nq, int k,
                float *__restrict__ od, int *__restrict__ oi) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<S, int> L;
    L.init();
    const int64_t total = (int64_t)nparts * k;
    for (int64_t c0 = 0; c0 < total; c0 += 64) {
        const int64_t c = c0 + lane;
        float key = __builtin_inff();
        int id = 0x7fffffff;
        if (c < total) {
            const int64_t p = c / k, i = c - p * k;
            const int64_t off = (p * nq + q) * k + i;
            if (pi[off] >= 0) { key = pd[off]; id = pi[off]; }
        }
        L.offer(key, id, k - 1);
    }
    L.store(od + q * k, oi + q * k, k);
}

// ---------------------------------------------------------------------------------------------
// Host launchers (called from hip_ann.cpp).
// ---------------------------------------------------------------------------------------------
void launch_row_norms(const float *x, int64_t n, int d, float *out, hipStream_t st) {
    if (n <= 0) return;
    const int vec4 = (d % 4 == 0) && ((uintptr_t)x % 16 == 0);
    hipLaunchKernelGGL(row_norms_f32, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, st, x, n, d, vec4, out);
    HIPANN_CHECK(hipGetLastError());
}

size_t gemm_smem_bytes() { return (size_t)4 * GBM * GLD * sizeof(float); }

void launch_flat_gemm_topk(const float *Q, const float *qn, int64_t nq, const float *X, const float *xn, int64_t N,
                           int d, int metric, int k, int nsplit, int64_t tiles_per_split, float *pd, int *pi,
                           hipStream_t st) {
    const int nqt = (int)ceil_div(nq, GBM);
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)Q % 16 == 0) && ((uintptr_t)X % 16 == 0);
    dim3 grid((unsigned)(nqt * nsplit)), block(256);
    static const int v1 = [] { const char *e = std::getenv("HIPANN_FLAT_V1"); return e ? std::atoi(e) : 0; }();
    if (!v1) {
        const size_t smem2 = gemm2_smem_bytes(k);
        if (metric == kL2) {
            if (vec4) hipLaunchKernelGGL((flat_gemm_topk2<true, true>), grid, block, smem2, st, Q, qn, nq, X, xn, N, d, k, nqt, nsplit, tiles_per_split, pd, pi);
            else hipLaunchKernelGGL((flat_gemm_topk2<false, true>), grid, block, smem2, st, Q, qn, nq, X, xn, N, d, k, nqt, nsplit, tiles_per_split, pd, pi);
        } else {
            if (vec4) hipLaunchKernelGGL((flat_gemm_topk2<true, false>), grid, block, smem2, st, Q, qn, nq, X, xn, N, d, k, nqt, nsplit, tiles_per_split, pd, pi);
            else hipLaunchKernelGGL((flat_gemm_topk2<false, false>), grid, block, smem2, st, Q, qn, nq, X, xn, N, d, k, nqt, nsplit, tiles_per_split, pd, pi);
        }
        HIPANN_CHECK(hipGetLastError());
        return;
    }
    const size_t smem = gemm_smem_bytes();
    if (vec4) {
        hipLaunchKernelGGL(flat_gemm_topk<true>, grid, block, smem, st, Q, qn, nq, X, xn, N, d, metric, k, nqt,
                           nsplit, tiles_per_split, pd, pi);
    } else {
        hipLaunchKernelGGL(flat_gemm_topk<false>, grid, block, smem, st, Q, qn, nq, X, xn, N, d, metric, k, nqt,
                           nsplit, tiles_per_split, pd, pi);
    }
    HIPANN_CHECK(hipGetLastError());
}

int flat_bf_dpad(int d) { return (d + GBK - 1) / GBK * GBK; }
size_t flat_bf_qsplit_bytes(int64_t nq, int d, int np) { return (size_t)nq * np * flat_bf_dpad(d) * 2; }

template <int NP>
static void launch_flat_gemm_topk_bf_t(const float *Q, const float *qn, int64_t nq, void *qsplit, const float *X,
                                       const float *xn, int64_t N, int d, int metric, int k, int nsplit,
                                       int64_t tiles_per_split, float *pd, int *pi, int qmajor, hipStream_t st) {
    const int dpad = flat_bf_dpad(d);
    const int64_t ng = nq * (dpad / 4);
    hipLaunchKernelGGL(flat_split_queries<NP>, dim3((unsigned)ceil_div(ng, 256)), dim3(256), 0, st, Q, nq, d, dpad,
                       reinterpret_cast<uint2 *>(qsplit));
    HIPANN_CHECK(hipGetLastError());
    // Block shape: 4 waves (128 queries, two blocks per CU) or 8 waves (256 queries, one block per CU, one
    // row staging shared by twice the MFMAs).  Measured at 10M × 768: 2 terms 60.3 ms (4) vs 65.6 ms (8),
    // 3 terms 90.6 ms (4) vs 86.2 ms (8).  HIPANN_FLAT_BF_WAVES=4|8 overrides (A/B).
    static const int Wenv = [] { const char *e = std::getenv("HIPANN_FLAT_BF_WAVES"); return e ? std::atoi(e) : 0; }();
    const int W = Wenv == 4 || Wenv == 8 ? Wenv : (NP == 3 ? 8 : 4);
    const int nqt = (int)ceil_div(nq, 32 * W);
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)X % 16 == 0);
    const size_t smem = gemm_bf_smem_bytes(NP, k, W);
    HIPANN_REQUIRE(smem <= 160 * 1024, "k too large for the split-bf16 Flat kernel");
    dim3 grid((unsigned)(nqt * nsplit)), block(64 * W);
    const uint4 *qs = reinterpret_cast<const uint4 *>(qsplit);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, smem, st, qs, dpad, qn, nq, X, xn, N, d, k, nqt, nsplit, tiles_per_split,
                           pd, pi, qmajor);
    };
    if (metric == kL2) {
        if (vec4) W == 8 ? go(flat_gemm_topk_bf<true, true, NP, 8>) : go(flat_gemm_topk_bf<true, true, NP, 4>);
        else W == 8 ? go(flat_gemm_topk_bf<false, true, NP, 8>) : go(flat_gemm_topk_bf<false, true, NP, 4>);
    } else {
        if (vec4) W == 8 ? go(flat_gemm_topk_bf<true, false, NP, 8>) : go(flat_gemm_topk_bf<true, false, NP, 4>);
        else W == 8 ? go(flat_gemm_topk_bf<false, false, NP, 8>) : go(flat_gemm_topk_bf<false, false, NP, 4>);
    }
    HIPANN_CHECK(hipGetLastError());
}

void launch_flat_gemm_topk_bf(int np, const float *Q, const float *qn, int64_t nq, void *qsplit, const float *X,
                              const float *xn, int64_t N, int d, int metric, int k, int nsplit, int64_t tiles_per_split,
                              float *pd, int *pi, int qmajor, hipStream_t st) {
    if (np == 2) launch_flat_gemm_topk_bf_t<2>(Q, qn, nq, qsplit, X, xn, N, d, metric, k, nsplit, tiles_per_split, pd, pi, qmajor, st);
    else launch_flat_gemm_topk_bf_t<3>(Q, qn, nq, qsplit, X, xn, N, d, metric, k, nsplit, tiles_per_split, pd, pi, qmajor, st);
}

// Key matrix of a small problem (the IVF coarse quantizer: 1024 queries × 1024 centroids gives the 128 × 128
// tiles of flat_gemm_topk only 64 blocks): 64 × 64 tiles, one 32 × 32 sub-tile per wave, the same fp32 MFMA
// in the same k order as flat_gemm_topk<WRITE> (bit-identical keys), 4× the blocks.
constexpr int SBM = 64;
template <bool VEC4>
__device__ __forceinline__ void small_stage_load(const float *__restrict__ base, int64_t row0, int64_t nrows, int d,
                                                 int k0, float4 (&r)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int f = threadIdx.x + 256 * p;  // float4 index within the 64×32 tile
        const int row = f >> 3, c4 = f & 7;
        const int64_t grow = row0 + row;
        const int kk = k0 + 4 * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (grow < nrows) {
            const float *src = base + grow * (int64_t)d + kk;
            if (VEC4) {
                if (kk < d) v = *reinterpret_cast<const float4 *>(src);
            } else {
                if (kk + 0 < d) v.x = src[0];
                if (kk + 1 < d) v.y = src[1];
                if (kk + 2 < d) v.z = src[2];
                if (kk + 3 < d) v.w = src[3];
            }
        }
        r[p] = v;
    }
}
__device__ __forceinline__ void small_stage_store(float *__restrict__ lds, const float4 (&r)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int f = threadIdx.x + 256 * p;
        *reinterpret_cast<float4 *>(lds + (f >> 3) * GLD + 4 * (f & 7)) = r[p];
    }
}

template <bool VEC4>
__global__ void __launch_bounds__(256)
flat_keys_small(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq, const float *__restrict__ X,
                const float *__restrict__ xnorm, int64_t N, int d, int metric, int nqt, float *__restrict__ keys_out,
                int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float As[2][SBM * GLD], Bs[2][SBM * GLD];
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = lb % nqt;
    const int64_t q0 = (int64_t)qt * SBM, x0 = (int64_t)(lb / nqt) * SBM;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int l31 = lane & 31, h = lane >> 5;
    const int nk = (d + GBK - 1) / GBK;
    // chunks kc+1 and kc+2 in flight in two register sets (set = chunk & 1) while chunk kc is multiplied:
    // the Q / centroid rows come from the Infinity Cache, ≈1 µs away — one chunk of lookahead (≈0.4 µs of
    // MFMAs) left every chunk waiting on its loads (32 µs for 1024 × 1024 × 768)
    float4 sa[2][2], sb[2][2];
    small_stage_load<VEC4>(Q, q0, nq, d, 0, sa[0]);
    small_stage_load<VEC4>(X, x0, N, d, 0, sb[0]);
    small_stage_store(As[0], sa[0]);
    small_stage_store(Bs[0], sb[0]);
    if (nk > 1) {
        small_stage_load<VEC4>(Q, q0, nq, d, GBK, sa[1]);
        small_stage_load<VEC4>(X, x0, N, d, GBK, sb[1]);
    }
    if (nk > 2) {
        small_stage_load<VEC4>(Q, q0, nq, d, 2 * GBK, sa[0]);
        small_stage_load<VEC4>(X, x0, N, d, 2 * GBK, sb[0]);
    }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    auto step = [&](int kc, auto par_c) {
        constexpr int P = decltype(par_c)::value;  // kc & 1
        const float *Ab = As[P], *Bb = Bs[P];
        // the chunk's 8 fragment reads first, then its 16 MFMAs (one LDS wait per chunk; same k order)
        f32x4 a4[4], b4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a4[u] = *reinterpret_cast<const f32x4 *>(Ab + (32 * wr + l31) * GLD + 16 * h + 4 * u);
            b4[u] = *reinterpret_cast<const f32x4 *>(Bb + (32 * wc + l31) * GLD + 16 * h + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[u][e], b4[u][e], acc, 0, 0, 0);
        if (kc + 1 < nk) {  // chunk kc+1 (register set 1−P) → LDS buffer 1−P, last read at kc−1
            small_stage_store(As[1 - P], sa[1 - P]);
            small_stage_store(Bs[1 - P], sb[1 - P]);
            if (kc + 3 < nk) {
                small_stage_load<VEC4>(Q, q0, nq, d, (kc + 3) * GBK, sa[1 - P]);
                small_stage_load<VEC4>(X, x0, N, d, (kc + 3) * GBK, sb[1 - P]);
            }
        }
        __syncthreads();
    };
    for (int kc = 0; kc < nk; kc += 2) {
        step(kc, std::integral_constant<int, 0>{});
        if (kc + 1 < nk) step(kc + 1, std::integral_constant<int, 1>{});
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t x = x0 + 32 * wc + l31;
        if (q < nq && x < N) {
            const float ip = acc[r];
            float key;
            if (metric == kL2) {
                key = fmaf(-2.f, ip, qnorm[q] + xnorm[x]);
                key = key < 0.f ? 0.f : key;
            } else {
                key = -ip;
            }
            keys_out[q * ldk + x] = key;
        }
    }
}

// flat_keys_ksplit — flat_keys_small's 64 × 64 tiles on 8 waves: waves 0-3 run the first half of the k
// chunks and waves 4-7 the second (each half its own two LDS buffers, the halves in lock step on the block
// barrier), then half 1 hands its accumulators to half 0 through LDS: key = f(acc₀ + acc₁).  Two waves per
// SIMD instead of one, so each SIMD's MFMA chain is half as long and the other wave hides its LDS reads and
// barrier waits.  Needs an even chunk count (d = 768: 12 + 12); the sum differs from the one-pass k order
// by the split (deterministic; the coarse keys are not bit-pinned to any CPU order).
template <bool VEC4>
__device__ __forceinline__ void ks_stage_load(const float *__restrict__ base, int64_t row0, int64_t nrows, int d, int k0,
                                              int t, float4 (&r)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int f = t + 256 * p;
        const int row = f >> 3, c4 = f & 7;
        const int64_t grow = row0 + row;
        const int kk = k0 + 4 * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (grow < nrows) {
            const float *src = base + grow * (int64_t)d + kk;
            if (VEC4) {
                if (kk < d) v = *reinterpret_cast<const float4 *>(src);
            } else {
                if (kk + 0 < d) v.x = src[0];
                if (kk + 1 < d) v.y = src[1];
                if (kk + 2 < d) v.z = src[2];
                if (kk + 3 < d) v.w = src[3];
            }
        }
        r[p] = v;
    }
}
__device__ __forceinline__ void ks_stage_store(float *__restrict__ lds, int t, const float4 (&r)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int f = t + 256 * p;
        *reinterpret_cast<float4 *>(lds + (f >> 3) * GLD + 4 * (f & 7)) = r[p];
    }
}

template <bool VEC4>
__global__ void __launch_bounds__(512)
flat_keys_ksplit(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq, const float *__restrict__ X,
                 const float *__restrict__ xnorm, int64_t N, int d, int metric, int nqt, float *__restrict__ keys_out,
                 int64_t ldk) {
    __shared__ __attribute__((aligned(16))) float As[2][2][SBM * GLD], Bs[2][2][SBM * GLD];
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = lb % nqt;
    const int64_t q0 = (int64_t)qt * SBM, x0 = (int64_t)(lb / nqt) * SBM;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int half = wave >> 2, t = threadIdx.x & 255;
    const int wr = (wave >> 1) & 1, wc = wave & 1;
    const int l31 = lane & 31, h = lane >> 5;
    const int nkh = ((d + GBK - 1) / GBK) >> 1;  // chunks per half (the launcher checks the count is even)
    const int kbase = half * nkh * GBK;
    float4 sa[2][2], sb[2][2];
    ks_stage_load<VEC4>(Q, q0, nq, d, kbase, t, sa[0]);
    ks_stage_load<VEC4>(X, x0, N, d, kbase, t, sb[0]);
    ks_stage_store(As[half][0], t, sa[0]);
    ks_stage_store(Bs[half][0], t, sb[0]);
    if (nkh > 1) {
        ks_stage_load<VEC4>(Q, q0, nq, d, kbase + GBK, t, sa[1]);
        ks_stage_load<VEC4>(X, x0, N, d, kbase + GBK, t, sb[1]);
    }
    if (nkh > 2) {
        ks_stage_load<VEC4>(Q, q0, nq, d, kbase + 2 * GBK, t, sa[0]);
        ks_stage_load<VEC4>(X, x0, N, d, kbase + 2 * GBK, t, sb[0]);
    }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    auto step = [&](int kc, auto par_c) {
        constexpr int P = decltype(par_c)::value;
        const float *Ab = As[half][P], *Bb = Bs[half][P];
        f32x4 a4[4], b4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a4[u] = *reinterpret_cast<const f32x4 *>(Ab + (32 * wr + l31) * GLD + 16 * h + 4 * u);
            b4[u] = *reinterpret_cast<const f32x4 *>(Bb + (32 * wc + l31) * GLD + 16 * h + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[u][e], b4[u][e], acc, 0, 0, 0);
        if (kc + 1 < nkh) {
            ks_stage_store(As[half][1 - P], t, sa[1 - P]);
            ks_stage_store(Bs[half][1 - P], t, sb[1 - P]);
            if (kc + 3 < nkh) {
                ks_stage_load<VEC4>(Q, q0, nq, d, kbase + (kc + 3) * GBK, t, sa[1 - P]);
                ks_stage_load<VEC4>(X, x0, N, d, kbase + (kc + 3) * GBK, t, sb[1 - P]);
            }
        }
        __syncthreads();
    };
    for (int kc = 0; kc < nkh; kc += 2) {
        step(kc, std::integral_constant<int, 0>{});
        if (kc + 1 < nkh) step(kc + 1, std::integral_constant<int, 1>{});
    }
    // half 1 → LDS (the tile buffers are free: every read finished before the last barrier) → half 0 adds
    float *xch = &As[0][0][0];
    if (half == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) xch[(r * 4 + (wave & 3)) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += xch[(r * 4 + wave) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t x = x0 + 32 * wc + l31;
        if (q < nq && x < N) {
            const float ip = acc[r];
            float key;
            if (metric == kL2) {
                key = fmaf(-2.f, ip, qnorm[q] + xnorm[x]);
                key = key < 0.f ? 0.f : key;
            } else {
                key = -ip;
            }
            keys_out[q * ldk + x] = key;
        }
    }
}

// flat_keys_bf3 — flat_keys_ksplit's tiles and K split (64 × 64 keys per block, waves 0-3 the first half of the
// 32-dim chunks, waves 4-7 the second, half 1's accumulators added by half 0 through LDS) with q·x on the bf16
// matrix cores: both operands are split while they are staged into LDS into three round-to-nearest bf16 terms
// (fb_split4: x = x₁ + x₂ + x₃ exactly for normal floats), and each 16-dim step runs flat_gemm_topk_bf's six term
// products (FbProducts<3>, smallest first; the dropped ones are ≤ 2⁻²⁶ relative) on v_mfma_f32_32x32x16_bf16
// with fp32 accumulation: fp32-level keys at 0.375 of the fp32 matrix-core time (the IVF coarse quantizer,
// HIPANN_COARSE_BF3).  LDS rows of 32 dims are 80 B (64 + 16 pad): a b128 fragment read by 16 lanes of 16
// consecutive rows touches 16 distinct 4-bank groups.  LDS: [half][buffer][term][64 query rows + 64 table rows]
// × 80 B = 120 KiB (one block per CU, as flat_keys_ksplit).
constexpr int KB3_ROW = 80;                 // bytes per staged row (32 bf16 + pad)
constexpr int KB3_TERM = 128 * KB3_ROW;     // one term of one buffer: 64 query rows then 64 table rows
constexpr int KB3_BUF = 3 * KB3_TERM;
__device__ __forceinline__ void kb3_stage_store(char *__restrict__ buf, int rowbase, int t, const float4 (&r)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int f = t + 256 * p;
        const int row = rowbase + (f >> 3), c4 = f & 7;
        uint2 o[3];
        fb_split4<3>(r[p], o);
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<uint2 *>(buf + j * KB3_TERM + row * KB3_ROW + 8 * c4) = o[j];
    }
}

template <bool VEC4, int NS>
__global__ void __launch_bounds__(512)
flat_keys_bf3(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq, const float *__restrict__ X,
              const float *__restrict__ xnorm, int64_t N, int d, int metric, int nqt, float *__restrict__ keys_out,
              int64_t ldk) {
    __shared__ __attribute__((aligned(16))) char lds[2 * 2 * KB3_BUF];
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = lb % nqt;
    const int64_t q0 = (int64_t)qt * SBM, x0 = (int64_t)(lb / nqt) * SBM;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int half = wave >> 2, t = threadIdx.x & 255;
    const int wr = (wave >> 1) & 1, wc = wave & 1;
    const int l31 = lane & 31, h = lane >> 5;
    const int nkh = ((d + GBK - 1) / GBK) >> 1;  // chunks per half (the launcher checks the count is even)
    const int kbase = half * nkh * GBK;
    char *hb = lds + half * 2 * KB3_BUF;  // this half's two buffers
    // NS chunks in flight in registers (set = chunk mod NS) ahead of the LDS buffer being multiplied (2: as
    // flat_keys_ksplit; deeper rings measured no faster, see the launcher)
    float4 sa[NS][2], sb[NS][2];
    ks_stage_load<VEC4>(Q, q0, nq, d, kbase, t, sa[0]);
    ks_stage_load<VEC4>(X, x0, N, d, kbase, t, sb[0]);
    kb3_stage_store(hb, 0, t, sa[0]);
    kb3_stage_store(hb, 64, t, sb[0]);
#pragma unroll
    for (int c = 1; c <= NS; ++c)
        if (c < nkh) {
            ks_stage_load<VEC4>(Q, q0, nq, d, kbase + c * GBK, t, sa[c % NS]);
            ks_stage_load<VEC4>(X, x0, N, d, kbase + c * GBK, t, sb[c % NS]);
        }
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // this lane's fragment offsets: query row 32·wr + l31 (A), table row 64 + 32·wc + l31 (B), dims 8h.. of each
    // 16-dim step s
    const int aoff = (32 * wr + l31) * KB3_ROW + 16 * h, boff = (64 + 32 * wc + l31) * KB3_ROW + 16 * h;
    // step kc (U = lcm(2, NS) consecutive steps unrolled: LDS buffer kc & 1, register set (kc + 1) mod NS)
    auto step = [&](int kc, auto u_c) __attribute__((always_inline)) {
        constexpr int U = decltype(u_c)::value;
        constexpr int P = U & 1, S1 = (U + 1) % NS;
        const char *b = hb + P * KB3_BUF;
        uint4 af[3][2], bf[3][2];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                af[j][s] = *reinterpret_cast<const uint4 *>(b + j * KB3_TERM + aoff + 32 * s);
                bf[j][s] = *reinterpret_cast<const uint4 *>(b + j * KB3_TERM + boff + 32 * s);
            }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int pr = 0; pr < FbProducts<3>::n; ++pr)
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(fb_bf16x8, af[FbProducts<3>::a(pr)][s]),
                                                              __builtin_bit_cast(fb_bf16x8, bf[FbProducts<3>::b(pr)][s]),
                                                              acc, 0, 0, 0);
        if (kc + 1 < nkh) {
            char *nb = hb + (1 - P) * KB3_BUF;
            kb3_stage_store(nb, 0, t, sa[S1]);
            kb3_stage_store(nb, 64, t, sb[S1]);
            if (kc + 1 + NS < nkh) {
                ks_stage_load<VEC4>(Q, q0, nq, d, kbase + (kc + 1 + NS) * GBK, t, sa[S1]);
                ks_stage_load<VEC4>(X, x0, N, d, kbase + (kc + 1 + NS) * GBK, t, sb[S1]);
            }
        }
        __syncthreads();
    };
    constexpr int UN = NS % 2 == 0 ? NS : 2 * NS;
    for (int kc = 0; kc < nkh; kc += UN) {
        [&]<int... U>(std::integer_sequence<int, U...>) __attribute__((always_inline)) {
            ((kc + U < nkh ? step(kc + U, std::integral_constant<int, U>{}) : void()), ...);
        }(std::make_integer_sequence<int, UN>{});
    }
    float *xch = reinterpret_cast<float *>(lds);
    if (half == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) xch[(r * 4 + (wave & 3)) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += xch[(r * 4 + wave) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t x = x0 + 32 * wc + l31;
        if (q < nq && x < N) {
            const float ip = acc[r];
            float key;
            if (metric == kL2) {
                key = fmaf(-2.f, ip, qnorm[q] + xnorm[x]);
                key = key < 0.f ? 0.f : key;
            } else {
                key = -ip;
            }
            keys_out[q * ldk + x] = key;
        }
    }
}

// flat_keys_direct — the same 64 × 64 tiles, MFMAs and k order as flat_keys_small (bit-identical keys), but every
// wave loads its own A / B fragments straight from memory into a 3-chunk register ring: no LDS staging, no
// per-chunk barrier.  The inputs are small and cache-resident (the coarse quantizer's queries and centroids),
// so the doubled L2 reads cost little, while the 4 waves — one per SIMD — no longer wait on each other
// (flat_keys_small: 32 µs for 1024 × 1024 × 768, ≈ 3× its MFMA time).
template <bool VEC4>
__device__ __forceinline__ void keys_frag_load(const float *__restrict__ base, int64_t row, int d, int k0,
                                               float4 (&r)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int kk = k0 + 4 * u;
        const float *src = base + row * (int64_t)d + kk;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (VEC4) {
            if (kk < d) v = *reinterpret_cast<const float4 *>(src);
        } else {
            if (kk + 0 < d) v.x = src[0];
            if (kk + 1 < d) v.y = src[1];
            if (kk + 2 < d) v.z = src[2];
            if (kk + 3 < d) v.w = src[3];
        }
        r[u] = v;
    }
}

template <bool VEC4, int KR>
__global__ void __launch_bounds__(256)
flat_keys_direct(const float *__restrict__ Q, const float *__restrict__ qnorm, int64_t nq, const float *__restrict__ X,
                 const float *__restrict__ xnorm, int64_t N, int d, int metric, int nqt, float *__restrict__ keys_out,
                 int64_t ldk) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int qt = lb % nqt;
    const int64_t q0 = (int64_t)qt * SBM, x0 = (int64_t)(lb / nqt) * SBM;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int l31 = lane & 31, h = lane >> 5;
    const int nk = (d + GBK - 1) / GBK;
    // this lane's fragment rows (rows past the end re-read the last row; their keys are never written)
    int64_t qa = q0 + 32 * wr + l31, xb = x0 + 32 * wc + l31;
    qa = qa < nq ? qa : nq - 1;
    xb = xb < N ? xb : N - 1;
    constexpr int R = KR;
    float4 ra[R][4], rb[R][4];
#pragma unroll
    for (int s = 0; s < R; ++s)
        if (s < nk) {
            keys_frag_load<VEC4>(Q, qa, d, s * GBK + 16 * h, ra[s]);
            keys_frag_load<VEC4>(X, xb, d, s * GBK + 16 * h, rb[s]);
        }
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    auto step = [&](int kc, auto slot_c) {
        constexpr int S = decltype(slot_c)::value;  // kc % R
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[S][u][e], rb[S][u][e], acc, 0, 0, 0);
        if (kc + R < nk) {
            keys_frag_load<VEC4>(Q, qa, d, (kc + R) * GBK + 16 * h, ra[S]);
            keys_frag_load<VEC4>(X, xb, d, (kc + R) * GBK + 16 * h, rb[S]);
        }
    };
    for (int kc = 0; kc < nk; kc += R) {
        [&]<int... P>(std::integer_sequence<int, P...>) {
            ((kc + P < nk ? step(kc + P, std::integral_constant<int, P>{}) : void()), ...);
        }(std::make_integer_sequence<int, R>{});
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t q = q0 + 32 * wr + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int64_t x = x0 + 32 * wc + l31;
        if (q < nq && x < N) {
            const float ip = acc[r];
            float key;
            if (metric == kL2) {
                key = fmaf(-2.f, ip, qnorm[q] + xnorm[x]);
                key = key < 0.f ? 0.f : key;
            } else {
                key = -ip;
            }
            keys_out[q * ldk + x] = key;
        }
    }
}

// Word copy between device memory and the device mapping of pinned host buffers (small host-pointer
// calls: no DMA-engine round trips for the query upload and the result download).
__global__ void __launch_bounds__(256) copy_words(const unsigned *__restrict__ src, unsigned *__restrict__ dst,
                                                  int64_t words) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

void launch_copy_words(const void *src, void *dst, size_t bytes, hipStream_t st) {
    HIPANN_REQUIRE(bytes % 4 == 0, "copy_words: bytes must be a multiple of 4");
    const int64_t words = (int64_t)(bytes / 4);
    if (words == 0) return;
    hipLaunchKernelGGL(copy_words, dim3((unsigned)std::min<int64_t>(64, ceil_div(words, 256))), dim3(256), 0, st,
                       static_cast<const unsigned *>(src), static_cast<unsigned *>(dst), words);
    HIPANN_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(64) post_words(const unsigned *__restrict__ src, unsigned *__restrict__ dst,
                                                 int words, unsigned token) {
    for (int i = threadIdx.x; i < words; i += 64) dst[i] = src[i];
    __threadfence_system();  // the words reach the host before the token does
    __syncthreads();         // every lane's words (one wave today; any block size stays ordered)
    if (threadIdx.x == 0) __hip_atomic_store(dst + words, token, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void *host_device_ptr(void *pinned) {
    void *p = nullptr;
    HIPANN_CHECK(hipHostGetDevicePointer(&p, pinned, 0));
    return p;
}

void launch_post_words(const void *src, void *host_dst, int words, unsigned token, hipStream_t st) {
    hipLaunchKernelGGL(post_words, dim3(1), dim3(64), 0, st, static_cast<const unsigned *>(src),
                       static_cast<unsigned *>(host_device_ptr(host_dst)), words, token);
    HIPANN_CHECK(hipGetLastError());
}

size_t scan_smem_bytes(int nq, int d);

void launch_flat_gemm_keys(const float *Q, const float *qn, int64_t nq, const float *X, const float *xn, int64_t N,
                           int d, int metric, float *keys, int64_t ldk, hipStream_t st, bool bf3) {
    const int nqt = (int)ceil_div(nq, GBM);
    const int64_t ntiles = ceil_div(N, GBN);
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)Q % 16 == 0) && ((uintptr_t)X % 16 == 0);
    if ((int64_t)nqt * ntiles < 512) {  // too few 128 × 128 tiles to fill the chip: 64 × 64
        const int sq = (int)ceil_div(nq, SBM);
        const int64_t blocks = (int64_t)sq * ceil_div(N, SBM);
        dim3 g((unsigned)blocks), b(256);
        // HIPANN_KEYS = 2 (default; even chunk counts): flat_keys_ksplit; 0 (and odd counts): LDS-staged
        // (flat_keys_small, 29.7 µs for 1024 × 1024 × 768); 3 / 6: the
        // register-ring flat_keys_direct with that many chunks in flight (A/B: 34.0 / 35.7 µs).  Measured and
        // dropped at r04: four K-groups of 4 waves (24.0 µs) and 64-dim stages (25.0 µs) against 23.9 µs.
        static const int mode = [] { const char *e = std::getenv("HIPANN_KEYS"); return e ? std::atoi(e) : 2; }();
        const int nk = (d + GBK - 1) / GBK;
        // the IVF coarse quantizer: the same tiles on the bf16 matrix cores (3 terms): 25.4 → 22.6-23.0 µs at 1024 ×
        // 1024 × 768.  Not the matrix cores' time (3.8 µs) and not the loads' depth: HIPANN_KEYS_DEPTH = 4 / 6 chunks
        // in flight (22.6 / 23.4 / 23.3 µs for 2 / 4 / 6) and two or four independent accumulator chains (22.8 / 22.6
        // vs 23.7 µs) were measured and left out; PMC: matrix cores busy ≈ 15 %, TD ≈ 33 %, TA ≈ 20 % of the kernel
        static const int depth = [] { const char *e = std::getenv("HIPANN_KEYS_DEPTH"); return e ? std::atoi(e) : 2; }();
        if (bf3 && nk % 2 == 0) {
#define HIPANN_KB3(NS)                                                                                                    \
    do {                                                                                                                \
        if (vec4) hipLaunchKernelGGL((flat_keys_bf3<true, NS>), g, dim3(512), 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk); \
        else hipLaunchKernelGGL((flat_keys_bf3<false, NS>), g, dim3(512), 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk); \
    } while (0)
            if (depth >= 4) HIPANN_KB3(4);
            else HIPANN_KB3(2);
#undef HIPANN_KB3
        } else if (mode == 2 && nk % 2 == 0) {  // default: the K-split tiles (8 waves, two per SIMD)
            if (vec4) hipLaunchKernelGGL(flat_keys_ksplit<true>, g, dim3(512), 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
            else hipLaunchKernelGGL(flat_keys_ksplit<false>, g, dim3(512), 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
        } else if (mode == 3) {
            if (vec4) hipLaunchKernelGGL((flat_keys_direct<true, 3>), g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
            else hipLaunchKernelGGL((flat_keys_direct<false, 3>), g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
        } else if (mode == 6) {
            if (vec4) hipLaunchKernelGGL((flat_keys_direct<true, 6>), g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
            else hipLaunchKernelGGL((flat_keys_direct<false, 6>), g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
        } else {
            if (vec4) hipLaunchKernelGGL(flat_keys_small<true>, g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
            else hipLaunchKernelGGL(flat_keys_small<false>, g, b, 0, st, Q, qn, nq, X, xn, N, d, metric, sq, keys, ldk);
        }
        HIPANN_CHECK(hipGetLastError());
        return;
    }
    const size_t smem = gemm_smem_bytes();
    dim3 grid((unsigned)(nqt * ntiles)), block(256);
    if (vec4)
        hipLaunchKernelGGL((flat_gemm_topk<true, true>), grid, block, smem, st, Q, qn, nq, X, xn, N, d, metric, 1, nqt,
                           (int)ntiles, (int64_t)1, nullptr, nullptr, keys, ldk);
    else
        hipLaunchKernelGGL((flat_gemm_topk<false, true>), grid, block, smem, st, Q, qn, nq, X, xn, N, d, metric, 1,
                           nqt, (int)ntiles, (int64_t)1, nullptr, nullptr, keys, ldk);
    HIPANN_CHECK(hipGetLastError());
}

template <int NQ>
static void scan_keys_dispatch(bool vec4, dim3 grid, size_t smem, hipStream_t st, const float *Q, const float *X,
                               int64_t N, int d, int metric, int64_t rpw, float *keys, int64_t ldk) {
    if (vec4)
        hipLaunchKernelGGL((flat_scan_topk<NQ, true, true>), grid, dim3(256), smem, st, Q, X, N, d, metric, 1, rpw,
                           nullptr, nullptr, keys, ldk);
    else
        hipLaunchKernelGGL((flat_scan_topk<NQ, false, true>), grid, dim3(256), smem, st, Q, X, N, d, metric, 1, rpw,
                           nullptr, nullptr, keys, ldk);
}

void launch_flat_scan_keys(const float *Q, int nq, const float *X, int64_t N, int d, int metric, float *keys,
                           int64_t ldk, hipStream_t st) {
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)X % 16 == 0);
    const size_t smem = scan_smem_bytes(nq, d);
    // ≥ 512 rows per wave on large tables, small ones spread over waves of ≥ 16 rows (as the fused scan)
    int64_t nwaves = std::min<int64_t>(8192, std::max<int64_t>(std::min<int64_t>(256, ceil_div(N, 16)),
                                                               ceil_div(N, 512)));
    const int64_t rpw = ceil_div(N, nwaves);
    nwaves = ceil_div(N, rpw);
    dim3 grid((unsigned)ceil_div(nwaves, 4));
    switch (nq) {
#define HIPANN_SCANK_CASE(n) \
    case n: scan_keys_dispatch<n>(vec4, grid, smem, st, Q, X, N, d, metric, rpw, keys, ldk); break;
        HIPANN_SCANK_CASE(1) HIPANN_SCANK_CASE(2) HIPANN_SCANK_CASE(3) HIPANN_SCANK_CASE(4) HIPANN_SCANK_CASE(5)
        HIPANN_SCANK_CASE(6) HIPANN_SCANK_CASE(7) HIPANN_SCANK_CASE(8) HIPANN_SCANK_CASE(9) HIPANN_SCANK_CASE(10)
        HIPANN_SCANK_CASE(11) HIPANN_SCANK_CASE(12) HIPANN_SCANK_CASE(13) HIPANN_SCANK_CASE(14) HIPANN_SCANK_CASE(15)
        HIPANN_SCANK_CASE(16) HIPANN_SCANK_CASE(17) HIPANN_SCANK_CASE(18) HIPANN_SCANK_CASE(19)
#undef HIPANN_SCANK_CASE
        default: throw HipError("flat_scan_keys: nq out of range");
    }
    HIPANN_CHECK(hipGetLastError());
}

void launch_rows_topk(const float *keys, int64_t ldk, int64_t ncols, int64_t nq, int64_t seg_len, int nseg, int k,
                      int id0, float *pd, int *pi, hipStream_t st) {
    const int S = (k + 63) / 64;
    dim3 grid((unsigned)ceil_div(nq * nseg, 4)), block(256);
#define HIPANN_ROWS_CASE(s)                                                                                       \
    if (S <= s) {                                                                                                 \
        hipLaunchKernelGGL(rows_topk<s>, grid, block, 0, st, keys, ldk, ncols, nq, seg_len, nseg, k, id0, pd, pi); \
        HIPANN_CHECK(hipGetLastError());                                                                          \
        return;                                                                                                   \
    }
    HIPANN_ROWS_CASE(1) HIPANN_ROWS_CASE(2) HIPANN_ROWS_CASE(4) HIPANN_ROWS_CASE(8) HIPANN_ROWS_CASE(16)
    HIPANN_ROWS_CASE(32)
#undef HIPANN_ROWS_CASE
    throw HipError("rows_topk: k too large");
}

// HIPANN_ROWSEL_WAVE=1: rows of 257..1024 keys on one wave (rows_select_small<16>) instead of a block (A/B)
static bool one_wave_rows() {
    static const bool v = [] { const char *e = std::getenv("HIPANN_ROWSEL_WAVE"); return e && std::atoi(e); }();
    return v;
}

bool launch_rows_select_out(const float *keys, int64_t ldk, int64_t ncols, int64_t nq, int k, int kout,
                            int64_t label_offset, float out_sign, float *D, int64_t *I, hipStream_t st,
                            IvfPlanHook *hook) {
    const int S = (kout + 63) / 64;
    if (S > 4 || ncols > 0x7ffffffe || k > kout) return false;  // the segment path + merge instead
    dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
    static const bool lists = [] { const char *e = std::getenv("HIPANN_ROWSEL_LIST"); return e && std::atoi(e); }();
    if (kout <= 64 && ncols <= 1024 && !lists) {  // rows of ≤ 1024 keys: the bitwise select
        const bool h = hook != nullptr;
        const int *ll = h ? hook->list_len : nullptr;
        const int nl = h ? hook->nlist : 0, cr = h ? hook->chunk_rows : 1;
        int *cc = h ? hook->ccnt : nullptr, *so = h ? hook->slot_off : nullptr, *qt = h ? hook->qtot : nullptr;
        // HIPANN_ROWSEL_NARROW=0 (A/B): rows of 257..1024 keys on the block select instead of the narrowed wave
        static const bool narrow = [] { const char *e = std::getenv("HIPANN_ROWSEL_NARROW"); return !e || std::atoi(e); }();
        if (ncols <= 256)
            hipLaunchKernelGGL(rows_select_small<4>, grid, block, 0, st, keys, ldk, (int)ncols, nq, k, kout,
                               label_offset, out_sign, D, I, ll, nl, cr, cc, so, qt);
        else if (narrow)
            hipLaunchKernelGGL(rows_select_narrow<16>, grid, block, 0, st, keys, ldk, (int)ncols, nq, k, kout,
                               label_offset, out_sign, D, I, ll, nl, cr, cc, so, qt);
        else if (!one_wave_rows())
            hipLaunchKernelGGL(rows_select_block, dim3((unsigned)nq), block, 0, st, keys, ldk, (int)ncols, nq, k, kout,
                               label_offset, out_sign, D, I, ll, nl, cr, cc, so, qt);
        else
            hipLaunchKernelGGL(rows_select_small<16>, grid, block, 0, st, keys, ldk, (int)ncols, nq, k, kout,
                               label_offset, out_sign, D, I, ll, nl, cr, cc, so, qt);
        HIPANN_CHECK(hipGetLastError());
        if (h) hook->done = true;
        return true;
    }
#define HIPANN_RSEL_CASE(s)                                                                                      \
    if (S <= s) {                                                                                                \
        hipLaunchKernelGGL(rows_select_out<s>, grid, block, 0, st, keys, ldk, ncols, nq, k, kout, label_offset, \
                           out_sign, D, I);                                                                      \
        HIPANN_CHECK(hipGetLastError());                                                                         \
        return true;                                                                                             \
    }
    HIPANN_RSEL_CASE(1) HIPANN_RSEL_CASE(2) HIPANN_RSEL_CASE(4)
#undef HIPANN_RSEL_CASE
    return false;
}

void launch_merge_raw(const float *pd, const int *pi, int nparts, int64_t nq, int k, float *od, int *oi,
                      hipStream_t st) {
    const int S = (k + 63) / 64;
    dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
#define HIPANN_MRAW_CASE(s)                                                                           \
    if (S <= s) {                                                                                     \
        hipLaunchKernelGGL(merge_parts_raw<s>, grid, block, 0, st, pd, pi, nparts, nq, k, od, oi);    \
        HIPANN_CHECK(hipGetLastError());                                                              \
        return;                                                                                       \
    }
    HIPANN_MRAW_CASE(1) HIPANN_MRAW_CASE(2) HIPANN_MRAW_CASE(4) HIPANN_MRAW_CASE(8) HIPANN_MRAW_CASE(16)
    HIPANN_MRAW_CASE(32)
#undef HIPANN_MRAW_CASE
    throw HipError("merge_raw: k too large");
}

template <int NQ>
static void scan_dispatch(bool vec4, dim3 grid, size_t smem, hipStream_t st, const float *Q, const float *X,
                          int64_t N, int d, int metric, int k, int64_t rpw, float *pd, int *pi) {
    if (vec4)
        hipLaunchKernelGGL((flat_scan_topk<NQ, true>), grid, dim3(256), smem, st, Q, X, N, d, metric, k, rpw, pd, pi);
    else
        hipLaunchKernelGGL((flat_scan_topk<NQ, false>), grid, dim3(256), smem, st, Q, X, N, d, metric, k, rpw, pd, pi);
}

size_t scan_smem_bytes(int nq, int d) { return (size_t)nq * ((d + 3) & ~3) * sizeof(float); }

void launch_flat_scan_topk(const float *Q, int nq, const float *X, int64_t N, int d, int metric, int k,
                           int nwaves, int64_t rows_per_wave, float *pd, int *pi, hipStream_t st) {
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)X % 16 == 0);
    const size_t smem = scan_smem_bytes(nq, d);
    dim3 grid((unsigned)ceil_div(nwaves, 4));
    switch (nq) {
#define HIPANN_SCAN_CASE(n) \
    case n: scan_dispatch<n>(vec4, grid, smem, st, Q, X, N, d, metric, k, rows_per_wave, pd, pi); break;
        HIPANN_SCAN_CASE(1) HIPANN_SCAN_CASE(2) HIPANN_SCAN_CASE(3) HIPANN_SCAN_CASE(4) HIPANN_SCAN_CASE(5)
        HIPANN_SCAN_CASE(6) HIPANN_SCAN_CASE(7) HIPANN_SCAN_CASE(8) HIPANN_SCAN_CASE(9) HIPANN_SCAN_CASE(10)
        HIPANN_SCAN_CASE(11) HIPANN_SCAN_CASE(12) HIPANN_SCAN_CASE(13) HIPANN_SCAN_CASE(14) HIPANN_SCAN_CASE(15)
        HIPANN_SCAN_CASE(16) HIPANN_SCAN_CASE(17) HIPANN_SCAN_CASE(18) HIPANN_SCAN_CASE(19)
#undef HIPANN_SCAN_CASE
        default: throw HipError("flat_scan_topk: nq out of range");
    }
    HIPANN_CHECK(hipGetLastError());
}

template <typename InId>
void launch_merge_parts(const float *pd, const InId *pi, int nparts, int64_t nq, int k, int kout,
                        int64_t label_offset, float in_sign, float out_sign, float *D, int64_t *I, hipStream_t st,
                        int64_t pstride_d, int64_t pstride_i) {
    if (nq <= 0) return;
    if (pstride_d < 0) pstride_d = nq * k;  // default layout [part][nq][k]
    if (pstride_i < 0) pstride_i = nq * k;
    dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
    const int S = (kout + 63) / 64;
#define HIPANN_MERGE_CASE(s)                                                                                  \
    if (S <= s) {                                                                                             \
        hipLaunchKernelGGL((merge_parts_topk<s, InId>), grid, block, 0, st, pd, pi, nparts, nq, k, kout, \
                           label_offset, in_sign, out_sign, D, I, pstride_d, pstride_i);                                    \
        HIPANN_CHECK(hipGetLastError());                                                                      \
        return;                                                                                               \
    }
    HIPANN_MERGE_CASE(1) HIPANN_MERGE_CASE(2) HIPANN_MERGE_CASE(4) HIPANN_MERGE_CASE(8) HIPANN_MERGE_CASE(16)
    HIPANN_MERGE_CASE(32)
#undef HIPANN_MERGE_CASE
    throw HipError("merge: k too large");
}

template <typename InId>
void launch_merge_parts_2level(const float *pd, const InId *pi, int nparts, int64_t nq, int k, int kout,
                               int64_t label_offset, float in_sign, float out_sign, float *D, int64_t *I, float *md,
                               long long *mi, int ngroups, hipStream_t st) {
    if (nq <= 0) return;
    HIPANN_REQUIRE(kout <= 64 && ngroups >= 1, "2-level merge: kout <= 64");
    const int ppg = (int)ceil_div(nparts, ngroups);
    ngroups = (int)ceil_div(nparts, ppg);
    hipLaunchKernelGGL((merge_parts_stage1<InId>), dim3((unsigned)ceil_div((int64_t)ngroups * nq, 4)), dim3(256), 0,
                       st, pd, pi, nparts, nq, k, kout, label_offset, in_sign, ppg, ngroups, md, mi);
    HIPANN_CHECK(hipGetLastError());
    hipLaunchKernelGGL(merge_groups_block, dim3((unsigned)nq), dim3(256), 0, st, md, mi, ngroups, nq, kout, out_sign, D,
                       I);
    HIPANN_CHECK(hipGetLastError());
}

template void launch_merge_parts_2level<int>(const float *, const int *, int, int64_t, int, int, int64_t, float, float,
                                             float *, int64_t *, float *, long long *, int, hipStream_t);

template void launch_merge_parts<int>(const float *, const int *, int, int64_t, int, int, int64_t, float, float,
                                      float *, int64_t *, hipStream_t, int64_t, int64_t);
template void launch_merge_parts<long long>(const float *, const long long *, int, int64_t, int, int, int64_t, float,
                                            float, float *, int64_t *, hipStream_t, int64_t, int64_t);

}  // namespace hipann
