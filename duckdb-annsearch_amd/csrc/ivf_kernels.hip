// ivf_kernels.hip — IVFFlat list-major scan for gfx950.
//
// Replaces MetalIndexIVFFlat::search (faiss-metal/src/MetalIndexIVFFlat.mm:122-256), which loops
// over queries on the host, gathers every probed list into fresh buffers per query and launches a
// GEMV-shaped distance + select per query.  Here the whole batch is one pipeline on one stream:
//
//   coarse quantizer  : the Flat kernels with k = nprobe  (FAISS quantizer->search, same nq<20 rule)
//   ivf_count         : histogram of (query, probe) pairs per list
//   ivf_plan          : one block — exclusive scans → bucket offsets and work-item offsets per list
//   ivf_fill          : scatter (query, probe) pairs into per-list buckets
//   ivf_scan_topk     : one block per work item = (list ℓ, ≤ 32 of the queries probing ℓ).  The
//                       list's rows stream through LDS ONCE per item (coalesced float4 loads), each
//                       of the 4 waves computes direct Σ(q−x)² (FAISS IVFFlat scans with fvec_L2sqr)
//                       for its 8 queries × 256 rows per tile and keeps one wave top-k list per query
//   merge_parts_topk  : per query, the k best of its nprobe partial lists (ids mapped to labels)
//
// HBM traffic per batch ≈ Σ_items |ℓ|·4d  (each list read once per 32 queries probing it) instead
// of Σ_queries Σ_probes |ℓ|·4d for the query-major reference.
#include "common.hpp"
#include "wave_topk.hpp"

namespace hipann {

constexpr int IVF_WAVES = 8;            // waves per work item (block)
constexpr int IVF_THREADS = 64 * IVF_WAVES;
constexpr int IVF_G = 32;               // queries per work item
constexpr int IVF_QW = IVF_G / IVF_WAVES;  // queries per wave
constexpr int IVF_TR = 256;             // list rows per tile (4 per lane)
constexpr int IVF_BK = 24;              // dims per LDS chunk
constexpr int IVF_LD = IVF_BK + 4;      // padded row stride: 28 dwords → 16 rows hit 16 distinct b128 slots
constexpr int IVF_CH = 2048;            // list rows per work item (big lists split into chunks)

__device__ __forceinline__ int ivf_nch(int len) { return (len + IVF_CH - 1) / IVF_CH; }

__global__ void ivf_count(const int64_t *__restrict__ probes, int64_t npairs, const int *__restrict__ list_len,
                          int nlist, int *__restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const int64_t l = probes[i];
    if (l < 0 || l >= nlist) return;
    if (list_len[l] <= 0) return;  // empty, or owned by another shard
    atomicAdd(cnt + l, 1);
}

// Single block: bucket_off[l] = Σ_{<l} cnt, item_off[l] = Σ_{<l} ceil(cnt/G)·nch(l) (one item per
// (query group, row chunk) of each list); cursor[l] = 0; total items in item_off[nlist].
__global__ void __launch_bounds__(1024) ivf_plan(const int *__restrict__ cnt, const int *__restrict__ list_len,
                                                 int nlist, int *__restrict__ bucket_off,
                                                 int *__restrict__ item_off, int *__restrict__ cursor) {
    __shared__ int sb[1024], si[1024];
    __shared__ int carry_b, carry_i;
    if (threadIdx.x == 0) { carry_b = 0; carry_i = 0; }
    __syncthreads();
    for (int base = 0; base < nlist; base += 1024) {
        const int l = base + threadIdx.x;
        const int c = l < nlist ? cnt[l] : 0;
        const int items = l < nlist ? ((c + IVF_G - 1) / IVF_G) * ivf_nch(list_len[l]) : 0;
        sb[threadIdx.x] = c;
        si[threadIdx.x] = items;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
            int vb = 0, vi = 0;
            if ((int)threadIdx.x >= o) { vb = sb[threadIdx.x - o]; vi = si[threadIdx.x - o]; }
            __syncthreads();
            sb[threadIdx.x] += vb;
            si[threadIdx.x] += vi;
            __syncthreads();
        }
        if (l < nlist) {
            bucket_off[l] = carry_b + sb[threadIdx.x] - c;
            item_off[l] = carry_i + si[threadIdx.x] - items;
            cursor[l] = 0;
        }
        __syncthreads();
        if (threadIdx.x == 1023) { carry_b += sb[1023]; carry_i += si[1023]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { bucket_off[nlist] = carry_b; item_off[nlist] = carry_i; }
}

__global__ void ivf_fill(const int64_t *__restrict__ probes, int64_t npairs, const int *__restrict__ list_len,
                         int nlist, const int *__restrict__ bucket_off, int *__restrict__ cursor,
                         int *__restrict__ bucket) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const int64_t l = probes[i];
    if (l < 0 || l >= nlist) return;
    if (list_len[l] <= 0) return;
    const int pos = atomicAdd(cursor + l, 1);
    bucket[bucket_off[l] + pos] = (int)i;  // pair index = q * nprobe + p
}

// Single block: partial-list slots.  Pair i (= q·nprobe + p, probing list l) owns nch(l) consecutive
// slots (one per row chunk of l; 0 if l is empty or not on this shard): slot_off = exclusive scan.
// The slots of one query are therefore the contiguous range [slot_off[q·np], slot_off[(q+1)·np]).
__global__ void __launch_bounds__(1024) ivf_slot_scan(const int64_t *__restrict__ probes, int64_t npairs,
                                                      const int *__restrict__ list_len, int nlist,
                                                      int *__restrict__ slot_off) {
    __shared__ int sv[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < npairs; base += 1024) {
        const int64_t i = base + threadIdx.x;
        int v = 0;
        if (i < npairs) {
            const int64_t l = probes[i];
            if (l >= 0 && l < nlist) v = ivf_nch(list_len[l]);
        }
        sv[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int t = 0;
            if ((int)threadIdx.x >= o) t = sv[threadIdx.x - o];
            __syncthreads();
            sv[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < npairs) slot_off[i] = carry + sv[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += sv[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) slot_off[npairs] = carry;
}

// Row staging: IVF_TR rows × IVF_BK dims = IVF_TR·IVF_BK/4 float4, IVF_SP per thread.
constexpr int IVF_F4 = IVF_BK / 4;                 // float4 per staged row segment
constexpr int IVF_SP = IVF_TR * IVF_F4 / IVF_THREADS;  // float4 staged per thread

template <bool VEC4>
__device__ __forceinline__ void ivf_stage_load(const float *__restrict__ codes, int64_t r0, int64_t r1, int d, int k0,
                                               float4 (&st)[IVF_SP]) {
#pragma unroll
    for (int p = 0; p < IVF_SP; ++p) {
        const int f = threadIdx.x + IVF_THREADS * p;
        const int row = f / IVF_F4, c4 = f - (f / IVF_F4) * IVF_F4;
        const int64_t gr = r0 + row;
        const int kk = k0 + 4 * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < r1) {
            const float *src = codes + gr * (int64_t)d + kk;
            if (VEC4) {
                if (kk < d) v = *reinterpret_cast<const float4 *>(src);
            } else {
                if (kk + 0 < d) v.x = src[0];
                if (kk + 1 < d) v.y = src[1];
                if (kk + 2 < d) v.z = src[2];
                if (kk + 3 < d) v.w = src[3];
            }
        }
        st[p] = v;
    }
}

__device__ __forceinline__ void ivf_stage_store(float *__restrict__ lds, const float4 (&st)[IVF_SP]) {
#pragma unroll
    for (int p = 0; p < IVF_SP; ++p) {
        const int f = threadIdx.x + IVF_THREADS * p;
        const int row = f / IVF_F4, c4 = f - (f / IVF_F4) * IVF_F4;
        *reinterpret_cast<float4 *>(lds + row * IVF_LD + 4 * c4) = st[p];
    }
}

// Query staging: thread t < IVF_G·IVF_F4 stages float4 (t % IVF_F4) of query slot t / IVF_F4.
template <bool VEC4>
__device__ __forceinline__ void ivf_stage_q(const float *__restrict__ Q, int qrow, int d, int k0, float4 &st) {
    const int t = threadIdx.x;
    const int kk = k0 + 4 * (t - (t / IVF_F4) * IVF_F4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (qrow >= 0) {
        const float *src = Q + (int64_t)qrow * d + kk;
        if (VEC4) {
            if (kk < d) v = *reinterpret_cast<const float4 *>(src);
        } else {
            if (kk + 0 < d) v.x = src[0];
            if (kk + 1 < d) v.y = src[1];
            if (kk + 2 < d) v.z = src[2];
            if (kk + 3 < d) v.w = src[3];
        }
    }
    st = v;
}

// One K chunk (IVF_BK dims) for NW queries × 4 rows per lane.  Query values are LDS broadcasts
// (wave-uniform address); row values are per-lane ds_read_b128.  Direct form: t = q − x, acc += t².
template <int NW, bool IP>
__device__ __forceinline__ void ivf_chunk(const float *__restrict__ cur, const float *__restrict__ qcur,
                                          float (&acc)[4][IVF_QW], int lane) {
#pragma unroll 1
    for (int u = 0; u < IVF_F4; ++u) {
        float4 xv[4], qv[NW];
#pragma unroll
        for (int r = 0; r < 4; ++r) xv[r] = *reinterpret_cast<const float4 *>(cur + (lane + 64 * r) * IVF_LD + 4 * u);
#pragma unroll
        for (int j = 0; j < NW; ++j) qv[j] = *reinterpret_cast<const float4 *>(qcur + j * IVF_LD + 4 * u);
#pragma unroll
        for (int j = 0; j < NW; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (IP) {
                    acc[r][j] = fmaf(qv[j].x, xv[r].x, acc[r][j]);
                    acc[r][j] = fmaf(qv[j].y, xv[r].y, acc[r][j]);
                    acc[r][j] = fmaf(qv[j].z, xv[r].z, acc[r][j]);
                    acc[r][j] = fmaf(qv[j].w, xv[r].w, acc[r][j]);
                } else {
                    float t;
                    t = qv[j].x - xv[r].x; acc[r][j] = fmaf(t, t, acc[r][j]);
                    t = qv[j].y - xv[r].y; acc[r][j] = fmaf(t, t, acc[r][j]);
                    t = qv[j].z - xv[r].z; acc[r][j] = fmaf(t, t, acc[r][j]);
                    t = qv[j].w - xv[r].w; acc[r][j] = fmaf(t, t, acc[r][j]);
                }
            }
        }
    }
}

// part_d / part_i: one k-list per slot (slot_off, above); part_i holds shard-local row numbers.
//
// Occupancy: LDS = 2·(IVF_TR + IVF_G)·IVF_LD·4 B = 64.5 KiB → 2 blocks of IVF_WAVES waves per CU
// (≤ 128 VGPRs at 8 waves: four waves per SIMD).  A lone wave can issue a VALU op only every 4
// cycles (MI355X_MICROARCH.md, "vector-instruction ISSUE cost"), and the per-K-chunk barrier and
// LDS/VMEM waits need other waves on the SIMD to cover them.
template <bool VEC4, bool IP>
__global__ void __launch_bounds__(IVF_THREADS, 2 * IVF_THREADS / 256)
ivf_scan_topk(const float *__restrict__ Q, int d, const float *__restrict__ codes, const int64_t *__restrict__ list_off,
              const int *__restrict__ cnt, const int *__restrict__ bucket_off, const int *__restrict__ item_off,
              const int *__restrict__ bucket, const int *__restrict__ slot_off, int nlist, int nprobe, int64_t nq,
              int k, float *__restrict__ part_d, int *__restrict__ part_i) {
    // LDS: x tiles [2][IVF_TR][IVF_LD] then query tiles [2][IVF_G][IVF_LD]
    extern __shared__ __attribute__((aligned(16))) float xs[];
    float *qs = xs + 2 * IVF_TR * IVF_LD;
    const int item = blockIdx.x;
    const int total = item_off[nlist];
    if (item >= total) return;
    // list owning this item: the last l with item_off[l] <= item (lists with no items share their
    // successor's offset)
    int lo = 0, hi = nlist - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (item_off[mid] <= item) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int64_t lr0 = list_off[l], lr1 = list_off[l + 1];
    const int nch = ivf_nch((int)(lr1 - lr0));
    const int rem = item - item_off[l];
    const int g = rem / nch, chunk = rem - g * nch;  // (query group, row chunk)
    // the list's c probing queries are split evenly over ng = ceil(c / G) groups
    const int c = cnt[l];
    const int ng = (c + IVF_G - 1) / IVF_G;
    const int q_begin = (int)((int64_t)g * c / ng), q_end = (int)((int64_t)(g + 1) * c / ng);
    const int nqi = q_end - q_begin;
    const int64_t r0 = lr0 + (int64_t)chunk * IVF_CH;
    const int64_t r1 = r0 + IVF_CH < lr1 ? r0 + IVF_CH : lr1;
    const int boff = bucket_off[l] + q_begin;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // this wave's query slots [wq0, wq0 + nwq): the group's queries split evenly over the 4 waves
    const int wq0 = __builtin_amdgcn_readfirstlane(wave * nqi / IVF_WAVES);
    const int nwq = __builtin_amdgcn_readfirstlane((wave + 1) * nqi / IVF_WAVES - wave * nqi / IVF_WAVES);

    // staging role: thread t stages query slot t / IVF_F4
    int qrow = -1;
    if (threadIdx.x < IVF_G * IVF_F4) {
        const int slot = threadIdx.x / IVF_F4;
        if (slot < nqi) qrow = bucket[boff + slot] / nprobe;
    }

    WaveList<1, int> lists[IVF_QW];
#pragma unroll
    for (int j = 0; j < IVF_QW; ++j) lists[j].init();

    const int nk = (d + IVF_BK - 1) / IVF_BK;
    float4 st[IVF_SP], sq;
    for (int64_t t0 = r0; t0 < r1; t0 += IVF_TR) {
        float acc[4][IVF_QW];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < IVF_QW; ++j) acc[r][j] = 0.f;

        ivf_stage_load<VEC4>(codes, t0, r1, d, 0, st);
        ivf_stage_q<VEC4>(Q, qrow, d, 0, sq);
        ivf_stage_store(xs, st);
        if (threadIdx.x < IVF_G * IVF_F4)
            *reinterpret_cast<float4 *>(qs + (threadIdx.x / IVF_F4) * IVF_LD + 4 * (threadIdx.x % IVF_F4)) = sq;
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const float *cur = xs + (kc & 1) * IVF_TR * IVF_LD;
            float *nxt = xs + ((kc + 1) & 1) * IVF_TR * IVF_LD;
            const float *qcur = qs + (kc & 1) * IVF_G * IVF_LD + wq0 * IVF_LD;
            float *qnxt = qs + ((kc + 1) & 1) * IVF_G * IVF_LD;
            if (kc + 1 < nk) {
                ivf_stage_load<VEC4>(codes, t0, r1, d, (kc + 1) * IVF_BK, st);
                ivf_stage_q<VEC4>(Q, qrow, d, (kc + 1) * IVF_BK, sq);
            }
            switch (nwq) {  // wave-uniform: one branch per K chunk, operand loads hoisted inside
                case 8: if constexpr (IVF_QW >= 8) ivf_chunk<8, IP>(cur, qcur, acc, lane); break;
                case 7: if constexpr (IVF_QW >= 7) ivf_chunk<7, IP>(cur, qcur, acc, lane); break;
                case 6: if constexpr (IVF_QW >= 6) ivf_chunk<6, IP>(cur, qcur, acc, lane); break;
                case 5: if constexpr (IVF_QW >= 5) ivf_chunk<5, IP>(cur, qcur, acc, lane); break;
                case 4: if constexpr (IVF_QW >= 4) ivf_chunk<4, IP>(cur, qcur, acc, lane); break;
                case 3: if constexpr (IVF_QW >= 3) ivf_chunk<3, IP>(cur, qcur, acc, lane); break;
                case 2: if constexpr (IVF_QW >= 2) ivf_chunk<2, IP>(cur, qcur, acc, lane); break;
                case 1: if constexpr (IVF_QW >= 1) ivf_chunk<1, IP>(cur, qcur, acc, lane); break;
                default: break;
            }
            if (kc + 1 < nk) {
                ivf_stage_store(nxt, st);
                if (threadIdx.x < IVF_G * IVF_F4)
                    *reinterpret_cast<float4 *>(qnxt + (threadIdx.x / IVF_F4) * IVF_LD + 4 * (threadIdx.x % IVF_F4)) = sq;
            }
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = t0 + lane + 64 * r;
            const bool v = row < r1;
#pragma unroll
            for (int j = 0; j < IVF_QW; ++j) {
                if (j < nwq) {
                    const float key = IP ? -acc[r][j] : acc[r][j];
                    lists[j].offer(v ? key : __builtin_inff(), v ? (int)row : 0x7fffffff, k - 1);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < IVF_QW; ++j) {
        if (j < nwq) {
            const int pr = bucket[boff + wq0 + j];
            const int64_t off = (int64_t)(slot_off[pr] + chunk) * k;
            lists[j].store(part_d + off, part_i + off, k);
        }
    }
}

// Merge each query's partial lists (its contiguous slot range), mapping shard-local rows to labels.
template <int S>
__global__ void __launch_bounds__(256)
ivf_merge_topk(const float *__restrict__ pd, const int *__restrict__ pi, const int64_t *__restrict__ ids,
               const int *__restrict__ slot_off, int nprobe, int64_t nq, int k, int kout, float out_sign,
               float *__restrict__ D, int64_t *__restrict__ I) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    WaveList<S, long long> L;
    L.init();
    const int64_t s0 = slot_off[q * nprobe], s1 = slot_off[(q + 1) * nprobe];
    const int64_t total = (s1 - s0) * k;
    for (int64_t c0 = 0; c0 < total; c0 += 64) {
        const int64_t c = c0 + lane;
        float key = __builtin_inff();
        long long lab = IdTraits<long long>::pad();
        if (c < total) {
            const int64_t off = s0 * k + c;
            const int raw = pi[off];
            const float v = pd[off];
            if (raw >= 0 && raw != 0x7fffffff && !(v == __builtin_inff())) {
                key = v;
                lab = (long long)ids[raw];
            }
        }
        L.offer(key, lab, kout - 1);
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

// ---------------------------------------------------------------------------------------------
void launch_ivf_plan(const int64_t *probes, int64_t nq, int nprobe, const int *list_len, int nlist, int *cnt,
                     int *bucket_off, int *item_off, int *cursor, int *bucket, int *slot_off, hipStream_t st) {
    const int64_t npairs = nq * nprobe;
    HIPANN_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)nlist, st));
    if (npairs > 0)
        hipLaunchKernelGGL(ivf_count, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, st, probes, npairs, list_len,
                           nlist, cnt);
    hipLaunchKernelGGL(ivf_plan, dim3(1), dim3(1024), 0, st, cnt, list_len, nlist, bucket_off, item_off, cursor);
    hipLaunchKernelGGL(ivf_slot_scan, dim3(1), dim3(1024), 0, st, probes, npairs, list_len, nlist, slot_off);
    if (npairs > 0)
        hipLaunchKernelGGL(ivf_fill, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, st, probes, npairs, list_len,
                           nlist, bucket_off, cursor, bucket);
    HIPANN_CHECK(hipGetLastError());
}

// Upper bound on work items given the largest list's chunk count.
// Σ_l ceil(cnt_l/G)·nch_l ≤ Σ_l (cnt_l/G + 1)·nch_l ≤ ceil(npairs/G)·max_nch + Σ_l nch_l.
int64_t ivf_max_items(int64_t nq, int nprobe, int nlist, int max_nch, int64_t nrows) {
    const int64_t npairs = nq * nprobe;
    return ceil_div(npairs, IVF_G) * std::max(max_nch, 1) + ceil_div(nrows, IVF_CH) + nlist;
}

int ivf_chunk_rows() { return IVF_CH; }

size_t ivf_scan_smem_bytes() { return (size_t)2 * (IVF_TR + IVF_G) * IVF_LD * sizeof(float); }

void launch_ivf_scan(const float *Q, int d, int metric, const float *codes, const int64_t *list_off, const int *cnt,
                     const int *bucket_off, const int *item_off, const int *bucket, const int *slot_off, int nlist,
                     int nprobe, int64_t nq, int k, int64_t max_items, float *pd, int *pi, hipStream_t st) {
    if (max_items <= 0) return;
    const bool vec4 = (d % 4 == 0) && ((uintptr_t)Q % 16 == 0) && ((uintptr_t)codes % 16 == 0);
    dim3 grid((unsigned)max_items), block(IVF_THREADS);
    const size_t smem = ivf_scan_smem_bytes();
#define HIPANN_IVF_LAUNCH(V, IPM)                                                                                    \
    hipLaunchKernelGGL((ivf_scan_topk<V, IPM>), grid, block, smem, st, Q, d, codes, list_off, cnt, bucket_off, item_off, \
                       bucket, slot_off, nlist, nprobe, nq, k, pd, pi)
    if (vec4) {
        if (metric == kIP) HIPANN_IVF_LAUNCH(true, true); else HIPANN_IVF_LAUNCH(true, false);
    } else {
        if (metric == kIP) HIPANN_IVF_LAUNCH(false, true); else HIPANN_IVF_LAUNCH(false, false);
    }
#undef HIPANN_IVF_LAUNCH
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_merge(const float *pd, const int *pi, const int64_t *ids, const int *slot_off, int nprobe, int64_t nq,
                      int k, int kout, float out_sign, float *D, int64_t *I, hipStream_t st) {
    if (nq <= 0) return;
    dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
    const int S = (kout + 63) / 64;
#define HIPANN_IVF_MERGE(s)                                                                                           \
    if (S <= s) {                                                                                                     \
        hipLaunchKernelGGL(ivf_merge_topk<s>, grid, block, 0, st, pd, pi, ids, slot_off, nprobe, nq, k, kout,       \
                           out_sign, D, I);                                                                           \
        HIPANN_CHECK(hipGetLastError());                                                                              \
        return;                                                                                                       \
    }
    HIPANN_IVF_MERGE(1) HIPANN_IVF_MERGE(2) HIPANN_IVF_MERGE(4) HIPANN_IVF_MERGE(8) HIPANN_IVF_MERGE(16)
    HIPANN_IVF_MERGE(32)
#undef HIPANN_IVF_MERGE
    throw HipError("ivf merge: k too large");
}

}  // namespace hipann
