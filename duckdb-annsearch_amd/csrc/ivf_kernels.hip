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

#include <algorithm>
#include <cstdlib>
#include <utility>

namespace hipann {

constexpr int IVF_WAVES = 8;            // waves per work item (block)
constexpr int IVF_THREADS = 64 * IVF_WAVES;
constexpr int IVF_G = 32;               // queries per work item
constexpr int IVF_QW = IVF_G / IVF_WAVES;  // queries per wave
constexpr int IVF_TR = 256;             // list rows per tile (4 per lane)
constexpr int IVF_BK = 24;              // dims per LDS chunk
constexpr int IVF_LD = IVF_BK + 4;      // padded row stride: 28 dwords → 16 rows hit 16 distinct b128 slots
#ifndef HIPANN_IVF_CH
#define HIPANN_IVF_CH 2048  // tuning builds: list rows per work item
#endif
constexpr int IVF_CH = HIPANN_IVF_CH;   // list rows per work item (big lists split into chunks)

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

// Single block: bucket_off[l] = Σ_{<l} cnt, item_off[l] = Σ_{<l} ceil(cnt/group)·nch(l) (one item per
// (query group, row chunk) of each list); cursor[l] = 0; total items in item_off[nlist].
__global__ void __launch_bounds__(1024) ivf_plan(const int *__restrict__ cnt, const int *__restrict__ list_len,
                                                 int nlist, int group, int *__restrict__ bucket_off,
                                                 int *__restrict__ item_off, int *__restrict__ cursor) {
    __shared__ int sb[1024], si[1024];
    __shared__ int carry_b, carry_i;
    if (threadIdx.x == 0) { carry_b = 0; carry_i = 0; }
    __syncthreads();
    for (int base = 0; base < nlist; base += 1024) {
        const int l = base + threadIdx.x;
        const int c = l < nlist ? cnt[l] : 0;
        const int items = l < nlist ? ivf_ngroups(c, group) * ivf_nch(list_len[l]) : 0;
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
__device__ __forceinline__ void slot_scan_block(const int64_t *__restrict__ probes, int64_t npairs,
                                                const int *__restrict__ list_len, int nlist, int *__restrict__ slot_off,
                                                int *wsum) {
    // Per round, wave w owns the contiguous pairs base + [1024w, 1024w + 1024) as 16 chunks of 64: lane
    // i of chunk j is pair 64j + i, so the 16 probe loads and the 16 list-length gathers of a lane are
    // coalesced across the wave and all independent (two memory latencies per round); each chunk is
    // then scanned with shuffles and the 16 wave totals are combined in LDS.  (The first version gave
    // each thread 32 consecutive pairs — strided loads — and a 10-step block scan: 43 µs at 32K pairs.)
    constexpr int J = 16;  // (32 spilled at 1024 threads per block)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int carry = 0;
    for (int64_t base = 0; base < npairs; base += 16 * 64 * J) {
        const int64_t seg = base + (int64_t)wave * 64 * J;
        int l[J];  // list ids fit 32 bits (64-bit ids spilled at 1024 threads per block)
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int64_t i = seg + 64 * j + lane;
            const int64_t pv = i < npairs ? probes[i] : -1;
            l[j] = pv >= 0 && pv < nlist ? (int)pv : -1;
        }
        int v[J];
#pragma unroll
        for (int j = 0; j < J; ++j) v[j] = l[j] >= 0 ? ivf_nch(list_len[l[j]]) : 0;
        int run = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            int x = v[j];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(x, o);
                if (lane >= o) x += t;
            }
            const int tot = __shfl(x, 63);
            v[j] = run + x - v[j];  // exclusive offset inside the wave's segment
            run += tot;
        }
        if (lane == 0) wsum[wave] = run;
        __syncthreads();
        int off = carry, total = 0;
        for (int w2 = 0; w2 < 16; ++w2) {
            const int t = wsum[w2];
            off += w2 < wave ? t : 0;
            total += t;
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int64_t i = seg + 64 * j + lane;
            if (i < npairs) slot_off[i] = off + v[j];
        }
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) slot_off[npairs] = carry;
}

__global__ void __launch_bounds__(1024) ivf_slot_scan(const int64_t *__restrict__ probes, int64_t npairs,
                                                      const int *__restrict__ list_len, int nlist,
                                                      int *__restrict__ slot_off) {
    __shared__ int wsum[16];
    slot_scan_block(probes, npairs, list_len, nlist, slot_off, wsum);
}

// Query-major plan (default): three launches, two of them wide.
//   ivf_count_q  — one wave per query: its pairs' list counts into ccnt (global atomics), the exclusive
//                  prefix of their slot counts within the query into slot_off, the query's total to qtot
//   ivf_plan_q   — one block: the list scans of ivf_plan (from ccnt, which it zeroes again for the next
//                  batch), the exclusive scan of qtot (query slot bases), slot_off[npairs], and the batch's
//                  other per-query state (the rerank's flag count, the scans' running bounds = +inf)
//   ivf_fill_q   — one wave per query: slot_off += the query's base, bucket fill
// (the list-major count / plan / slot scan / fill sequence kept a 1024-pair single block on one CU for
// the slot scan: ≈ 55 µs of a 1024-query batch)
__global__ void __launch_bounds__(256) ivf_count_q(const int64_t *__restrict__ probes, int64_t nq, int nprobe,
                                                   const int *__restrict__ list_len, int nlist, int *__restrict__ ccnt,
                                                   int *__restrict__ slot_off, int *__restrict__ qtot) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    int carry = 0;
    for (int p0 = 0; p0 < nprobe; p0 += 64) {
        const int p = p0 + lane;
        const int64_t i = q * nprobe + p;
        const int64_t l = p < nprobe ? probes[i] : -1;
        const bool ok = l >= 0 && l < nlist;
        const int len = ok ? list_len[l] : 0;
        if (len > 0) atomicAdd(ccnt + (int64_t)(q % kPlanCopies) * nlist + l, 1);
        const int v = len > 0 ? ivf_nch(len) : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o);
            if (lane >= o) x += t;
        }
        if (p < nprobe) slot_off[i] = carry + x - v;
        carry += __shfl(x, 63);
    }
    if (lane == 0) qtot[q] = carry;
}

__global__ void __launch_bounds__(1024) ivf_plan_q(int *__restrict__ ccnt, const int *__restrict__ list_len, int nlist,
                                                   int group, int *__restrict__ cnt, int *__restrict__ bucket_off,
                                                   int *__restrict__ item_off, int *__restrict__ cursor,
                                                   int *__restrict__ qtot, int64_t nq, int64_t npairs,
                                                   int *__restrict__ slot_off, int *__restrict__ nflag_reset,
                                                   unsigned *__restrict__ qbound) {
    __shared__ int sb[1024], si[1024];
    __shared__ int carry_b, carry_i;
    const int tid = threadIdx.x;
    if (tid == 0) { carry_b = 0; carry_i = 0; }
    if (nflag_reset && tid == 0) *nflag_reset = 0;
    if (qbound)
        for (int64_t q = tid; q < nq; q += 1024) qbound[q] = 0xff800000u;
    __syncthreads();
    for (int base = 0; base < nlist; base += 1024) {
        const int l = base + tid;
        int c = 0;
        if (l < nlist)
            for (int cp = 0; cp < kPlanCopies; ++cp) c += ccnt[(int64_t)cp * nlist + l];
        const int items = l < nlist ? ivf_ngroups(c, group) * ivf_nch(list_len[l]) : 0;
        sb[tid] = c;
        si[tid] = items;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
            int vb = 0, vi = 0;
            if (tid >= o) { vb = sb[tid - o]; vi = si[tid - o]; }
            __syncthreads();
            sb[tid] += vb;
            si[tid] += vi;
            __syncthreads();
        }
        if (l < nlist) {
            cnt[l] = c;
            bucket_off[l] = carry_b + sb[tid] - c;
            item_off[l] = carry_i + si[tid] - items;
            int pre = 0;  // copy cp's fills start after copies 0..cp-1 (ivf_fill_q adds to its copy's cursor)
            for (int cp = 0; cp < kPlanCopies; ++cp) {
                const int64_t e = (int64_t)cp * nlist + l;
                const int n = ccnt[e];
                cursor[e] = pre;
                ccnt[e] = 0;
                pre += n;
            }
        }
        __syncthreads();
        if (tid == 1023) { carry_b += sb[1023]; carry_i += si[1023]; }
        __syncthreads();
    }
    if (tid == 0) { bucket_off[nlist] = carry_b; item_off[nlist] = carry_i; }
    // query slot bases: exclusive scan of qtot, in place
    __syncthreads();
    if (tid == 0) carry_b = 0;
    __syncthreads();
    for (int64_t base = 0; base < nq; base += 1024) {
        const int64_t q = base + tid;
        const int t = q < nq ? qtot[q] : 0;
        sb[tid] = t;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int v = 0;
            if (tid >= o) v = sb[tid - o];
            __syncthreads();
            sb[tid] += v;
            __syncthreads();
        }
        if (q < nq) qtot[q] = carry_b + sb[tid] - t;
        __syncthreads();
        if (tid == 1023) carry_b += sb[1023];
        __syncthreads();
    }
    if (tid == 0) slot_off[npairs] = carry_b;
}

__global__ void __launch_bounds__(256) ivf_fill_q(const int64_t *__restrict__ probes, int64_t nq, int nprobe,
                                                  const int *__restrict__ list_len, int nlist,
                                                  const int *__restrict__ qbase, const int *__restrict__ bucket_off,
                                                  int *__restrict__ cursor, int *__restrict__ bucket,
                                                  int *__restrict__ slot_off) {
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    const int b = qbase[q];
    for (int p = lane; p < nprobe; p += 64) {
        const int64_t i = q * nprobe + p;
        slot_off[i] += b;
        const int64_t l = probes[i];
        if (l < 0 || l >= nlist || list_len[l] <= 0) continue;
        const int pos = atomicAdd(cursor + (int64_t)(q % kPlanCopies) * nlist + l, 1);
        bucket[bucket_off[l] + pos] = (int)i;
    }
}

// ivf_planfill_q — ivf_plan_q and ivf_fill_q in one launch (nlist ≤ kPlanFillMaxList): every block recomputes
// the two prefixes it needs from the counts — the lists' bucket offsets (nlist values) and its queries' slot
// bases (a sum over the preceding queries' totals) — instead of waiting for a one-block scan; block 0
// publishes the scan's tables (cnt, bucket_off, item_off, the slot total) and the batch's resets.  The
// per-list counts and fill cursors are double-buffered by batch parity: this batch reads ccnt / cursor (zero
// on entry) and zeroes the other pair for the next batch (its count step runs after this kernel).
constexpr int kPlanFillMaxList = 8192;
__device__ __forceinline__ int block_excl_scan256(int v, int *s_w) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(x, o);
        if (lane >= o) x += t;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) base += w < wave ? s_w[w] : 0;
    __syncthreads();
    return base + x - v;
}
__global__ void __launch_bounds__(256) ivf_planfill_q(const int64_t *__restrict__ probes, int64_t nq, int nprobe,
                                                      const int *__restrict__ list_len, int nlist, int group,
                                                      const int *__restrict__ ccnt, int *__restrict__ ccnt_next,
                                                      int *__restrict__ cursor, int *__restrict__ cursor_next,
                                                      const int *__restrict__ qtot, int *__restrict__ slot_off,
                                                      int64_t npairs, int *__restrict__ cnt, int *__restrict__ bucket_off,
                                                      int *__restrict__ item_off, int *__restrict__ bucket,
                                                      int *__restrict__ nflag_reset, unsigned *__restrict__ qbound) {
    __shared__ int s_boff[kPlanFillMaxList];
    __shared__ int s_w[4], s_qb[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t q0 = (int64_t)blockIdx.x * 4;
    // list bucket offsets: thread t owns lists [t·per, (t+1)·per)
    const int per = (nlist + 255) / 256;
    int sum = 0, isum = 0;
    for (int j = 0; j < per; ++j) {
        const int l = tid * per + j;
        if (l < nlist) {
            int c = 0;
            for (int cp = 0; cp < kPlanCopies; ++cp) c += ccnt[(int64_t)cp * nlist + l];
            sum += c;
            if (blockIdx.x == 0) isum += ivf_ngroups(c, group) * ivf_nch(list_len[l]);
        }
    }
    int b = block_excl_scan256(sum, s_w);
    int ib = blockIdx.x == 0 ? block_excl_scan256(isum, s_w) : 0;
    for (int j = 0; j < per; ++j) {
        const int l = tid * per + j;
        if (l < nlist) {
            int c = 0;
            for (int cp = 0; cp < kPlanCopies; ++cp) c += ccnt[(int64_t)cp * nlist + l];
            s_boff[l] = b;
            if (blockIdx.x == 0) {
                cnt[l] = c;
                bucket_off[l] = b;
                item_off[l] = ib;
                ib += ivf_ngroups(c, group) * ivf_nch(list_len[l]);
            }
            b += c;
        }
    }
    if (blockIdx.x == 0 && tid == 255) {
        bucket_off[nlist] = b;
        item_off[nlist] = ib;
    }
    // the next batch's counts and cursors start at zero (each block clears a slice)
    for (int64_t l = (int64_t)blockIdx.x * 256 + tid; l < (int64_t)kPlanCopies * nlist; l += (int64_t)gridDim.x * 256) {
        ccnt_next[l] = 0;
        cursor_next[l] = 0;
    }
    // this block's queries' slot bases: Σ qtot over the preceding queries
    int qs = 0;
    for (int64_t q = tid; q < q0; q += 256) qs += qtot[q];
    const int qb0 = block_excl_scan256(qs, s_w) + qs;  // the block-wide total (inclusive of the last thread)
    if (tid == 255) s_qb[0] = qb0;
    __syncthreads();
    if (tid == 0) {
        int acc = s_qb[0];
        for (int i = 0; i < 4; ++i) {
            s_qb[i] = acc;
            acc += q0 + i < nq ? qtot[q0 + i] : 0;
        }
        if (q0 + 4 >= nq) slot_off[npairs] = acc;  // the last block: every query's slots
        if (blockIdx.x == 0 && nflag_reset) *nflag_reset = 0;
    }
    __syncthreads();
    // fill (one wave per query): slot_off += the query's base, bucket
    const int64_t q = q0 + wave;
    if (q >= nq) return;
    if (qbound && lane == 0) qbound[q] = 0xff800000u;
    const int base = s_qb[wave];
    for (int p = lane; p < nprobe; p += 64) {
        const int64_t i = q * nprobe + p;
        slot_off[i] += base;
        const int64_t l = probes[i];
        if (l < 0 || l >= nlist || list_len[l] <= 0) continue;
        // this query's copy of the list's cursor; its rows follow copies 0..cp-1 in the list's bucket
        const int cp = (int)(q % kPlanCopies);
        int pre = 0;
        for (int c2 = 0; c2 < cp; ++c2) pre += ccnt[(int64_t)c2 * nlist + l];
        const int pos = atomicAdd(cursor + (int64_t)cp * nlist + l, 1);
        bucket[s_boff[l] + pre + pos] = (int)i;
    }
}

// Row staging: IVF_TR rows × IVF_BK dims = IVF_TR·IVF_BK/4 float4, IVF_SP per thread.
constexpr int IVF_F4 = IVF_BK / 4;                     // float4 per staged row segment
constexpr int IVF_SP = IVF_TR * IVF_F4 / IVF_THREADS;  // float4 staged per thread

// Branch-free staging: rows past the chunk re-load the chunk's last row (their results are never
// offered) and query slots past the group re-load its first query, so no load is predicated on the
// row; only VEC4 == false (d % 4 != 0 or unaligned) pays per-element bounds checks.
template <bool VEC4>
__device__ __forceinline__ float4 ivf_ld4(const float *__restrict__ src, int kk, int d) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (VEC4) {
        if (kk < d) v = *reinterpret_cast<const float4 *>(src);
    } else {
        if (kk + 0 < d) v.x = src[0];
        if (kk + 1 < d) v.y = src[1];
        if (kk + 2 < d) v.z = src[2];
        if (kk + 3 < d) v.w = src[3];
    }
    return v;
}

template <bool VEC4>
__device__ __forceinline__ void ivf_stage_load(const float *__restrict__ codes, int64_t r0, int64_t rlast, int d,
                                               int k0, float4 (&st)[IVF_SP]) {
#pragma unroll
    for (int p = 0; p < IVF_SP; ++p) {
        const int f = threadIdx.x + IVF_THREADS * p;
        const int row = f / IVF_F4, c4 = f - (f / IVF_F4) * IVF_F4;
        const int64_t gr = r0 + row < rlast ? r0 + row : rlast;
        const int kk = k0 + 4 * c4;
        st[p] = ivf_ld4<VEC4>(codes + gr * (int64_t)d + kk, kk, d);
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

// One K chunk (IVF_BK dims) for NW queries × 4 rows per lane.  Query values are LDS broadcasts
// (wave-uniform address); row values are per-lane ds_read_b128.  Direct form on packed f32 pairs
// (v_pk_add_f32 / v_pk_fma_f32, the only way to the 64 FLOP/clk/SIMD f32 VALU rate): each (row,
// query) accumulates even and odd dimensions in the two halves of a float2, summed at the end —
// a 2-way split of the sum, as FAISS's own SIMD fvec_L2sqr splits it 8 ways.
typedef float ivf_f2 __attribute__((ext_vector_type(2)));
typedef float ivf_f4 __attribute__((ext_vector_type(4)));

// a − b on a packed pair.  The backend splits a v2f32 fsub into two v_sub_f32 (and folds
// fma(b, −1, a) back into that fsub), so the packed form is spelled out.
__device__ __forceinline__ ivf_f2 ivf_pk_sub(ivf_f2 a, ivf_f2 b) {
    ivf_f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int NW, bool IP>
__device__ __forceinline__ void ivf_chunk(const float *__restrict__ cur, const float *__restrict__ qcur,
                                          ivf_f2 (&acc)[4][NW > 0 ? NW : 1], int lane) {
#pragma unroll 1
    for (int u = 0; u < IVF_F4; ++u) {
        ivf_f4 xv[4], qv[NW > 0 ? NW : 1];
#pragma unroll
        for (int r = 0; r < 4; ++r) xv[r] = *reinterpret_cast<const ivf_f4 *>(cur + (lane + 64 * r) * IVF_LD + 4 * u);
#pragma unroll
        for (int j = 0; j < NW; ++j) qv[j] = *reinterpret_cast<const ivf_f4 *>(qcur + j * IVF_LD + 4 * u);
#pragma unroll
        for (int j = 0; j < NW; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (IP) {
                    acc[r][j] = __builtin_elementwise_fma(qv[j].xy, xv[r].xy, acc[r][j]);
                    acc[r][j] = __builtin_elementwise_fma(qv[j].zw, xv[r].zw, acc[r][j]);
                } else {
                    ivf_f2 t = ivf_pk_sub(qv[j].xy, xv[r].xy);
                    acc[r][j] = __builtin_elementwise_fma(t, t, acc[r][j]);
                    t = ivf_pk_sub(qv[j].zw, xv[r].zw);
                    acc[r][j] = __builtin_elementwise_fma(t, t, acc[r][j]);
                }
            }
        }
    }
}

// The whole (list chunk × query group) item for a wave owning NW query slots (NW may be 0: the wave
// still stages and meets every barrier).  Every wave of the block runs the same tile / K loop trip
// counts, so the barriers line up across waves with different NW.
template <int NW, bool VEC4, bool IP>
__device__ __forceinline__ void ivf_scan_item(const float *__restrict__ Q, int d, const float *__restrict__ codes,
                                              int64_t r0, int64_t r1, int qrow, int wq0, const int *__restrict__ bucket,
                                              int boff, const int *__restrict__ slot_off, int chunk, int k,
                                              float *__restrict__ xs, float *__restrict__ qs,
                                              float *__restrict__ part_d, int *__restrict__ part_i) {
    constexpr int NA = NW > 0 ? NW : 1;
    const int lane = threadIdx.x & 63;
    const bool qstager = threadIdx.x < IVF_G * IVF_F4;
    const int qslot = threadIdx.x / IVF_F4, qc4 = threadIdx.x - (threadIdx.x / IVF_F4) * IVF_F4;
    const float *qsrc = Q + (int64_t)qrow * d;
    WaveList<1, int> lists[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) lists[j].init();

    const int nk = (d + IVF_BK - 1) / IVF_BK;
    float4 st[IVF_SP], sq = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t t0 = r0; t0 < r1; t0 += IVF_TR) {
        ivf_f2 acc[4][NA];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < NA; ++j) acc[r][j] = ivf_f2{0.f, 0.f};

        ivf_stage_load<VEC4>(codes, t0, r1 - 1, d, 0, st);
        if (qstager) sq = ivf_ld4<VEC4>(qsrc + 4 * qc4, 4 * qc4, d);
        ivf_stage_store(xs, st);
        if (qstager) *reinterpret_cast<float4 *>(qs + qslot * IVF_LD + 4 * qc4) = sq;
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const float *cur = xs + (kc & 1) * IVF_TR * IVF_LD;
            float *nxt = xs + ((kc + 1) & 1) * IVF_TR * IVF_LD;
            const float *qcur = qs + (kc & 1) * IVF_G * IVF_LD + wq0 * IVF_LD;
            float *qnxt = qs + ((kc + 1) & 1) * IVF_G * IVF_LD;
            const bool more = kc + 1 < nk;
            if (more) {
                const int k1 = (kc + 1) * IVF_BK;
                ivf_stage_load<VEC4>(codes, t0, r1 - 1, d, k1, st);
                if (qstager) sq = ivf_ld4<VEC4>(qsrc + k1 + 4 * qc4, k1 + 4 * qc4, d);
            }
            if (NW > 0) ivf_chunk<NW, IP>(cur, qcur, acc, lane);
            if (more) {
                ivf_stage_store(nxt, st);
                if (qstager) *reinterpret_cast<float4 *>(qnxt + qslot * IVF_LD + 4 * qc4) = sq;
            }
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t row = t0 + lane + 64 * r;
            const bool v = row < r1;
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const float sum = acc[r][j].x + acc[r][j].y;
                const float key = IP ? -sum : sum;
                lists[j].offer(v ? key : __builtin_inff(), v ? (int)row : 0x7fffffff, k - 1);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const int pr = bucket[boff + wq0 + j];
        const int64_t off = (int64_t)(slot_off[pr] + chunk) * k;
        lists[j].store(part_d + off, part_i + off, k);
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
ivf_scan_topk(const float *__restrict__ Q, int d, const float *__restrict__ codes, const int64_t *__restrict__ list_off, const int *__restrict__ list_len,
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
    const int64_t lr0 = list_off[l], lr1 = lr0 + list_len[l];
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

    const int wave = threadIdx.x >> 6;
    // this wave's query slots [wq0, wq0 + nwq): the group's queries split evenly over the waves
    const int wq0 = __builtin_amdgcn_readfirstlane(wave * nqi / IVF_WAVES);
    const int nwq = __builtin_amdgcn_readfirstlane((wave + 1) * nqi / IVF_WAVES - wave * nqi / IVF_WAVES);
    // staging role: thread t stages query slot t / IVF_F4 (slots past the group re-load slot 0)
    int qrow = 0;
    if (threadIdx.x < IVF_G * IVF_F4) {
        const int slot = threadIdx.x / IVF_F4;
        qrow = bucket[boff + (slot < nqi ? slot : 0)] / nprobe;
    }
    switch (nwq) {
        case 0: ivf_scan_item<0, VEC4, IP>(Q, d, codes, r0, r1, qrow, wq0, bucket, boff, slot_off, chunk, k, xs, qs, part_d, part_i); break;
        case 1: ivf_scan_item<1, VEC4, IP>(Q, d, codes, r0, r1, qrow, wq0, bucket, boff, slot_off, chunk, k, xs, qs, part_d, part_i); break;
        case 2: ivf_scan_item<2, VEC4, IP>(Q, d, codes, r0, r1, qrow, wq0, bucket, boff, slot_off, chunk, k, xs, qs, part_d, part_i); break;
        case 3: ivf_scan_item<3, VEC4, IP>(Q, d, codes, r0, r1, qrow, wq0, bucket, boff, slot_off, chunk, k, xs, qs, part_d, part_i); break;
        default: ivf_scan_item<IVF_QW, VEC4, IP>(Q, d, codes, r0, r1, qrow, wq0, bucket, boff, slot_off, chunk, k, xs, qs, part_d, part_i); break;
    }
}

// ---------------------------------------------------------------------------------------------
// ivf_scan_dot — the decomposed form ‖q‖² + ‖x‖² − 2·q·x (clamped ≥ 0; IP: q·x), as faiss-metal's
// IVF path and FAISS's GPU IVFFlat compute it (norms stored with the lists, MetalIndexIVFFlat.mm:
// 305-318).  One FMA per (query, row, dim) instead of the direct form's subtract + FMA, so the
// VALU floor halves; the kernel is register-blocked to keep LDS traffic below the FMA rate.
//
// Work item and outputs as ivf_scan_topk (same plan and slots, IVF_CH-row chunks, but groups of
// ≤ DT_G = 64 queries), items ordered
// (list, row chunk, query group) with the group fastest and dealt XCD-contiguously, so the groups
// that re-read one row chunk run together on one XCD and share its L2.
//
// Block: 4 waves, 2 blocks per CU.  Wave w owns ≤ DT_NW = 16 of the item's ≤ DT_G = 64 queries
// (so a list probed by up to 64 queries of the batch is streamed once) and every row of the tile:
// DT_R = 4 rows per lane (tile = 256 rows); per 4-dim step it reads its 4 rows' float4 once and
// applies them to its queries in blocks of ≤ 8 (8 broadcast ds_read_b128 + 128 FMAs per block).
//
// Staging: LDS-DMA (global_load_lds_dwordx4) into two stages, one chunk in flight while the other
// is read.  A chunk is DT_BK = 32 dims = one whole 128-B line of each row, so every line is fetched
// by one chunk of one item (12-dim chunks, whose lines span three chunks, were re-fetched after the
// XCD's L2 had streamed other blocks' rows through: 2× FETCH_SIZE).  Stage image: x = [256 rows]
// [8 float4] with the float4 index XOR-swizzled by (row >> 1) & 7 (applied on the DMA's per-lane
// SOURCE address — the DMA destination is lane-linear) so that the per-lane ds_read_b128 of 16
// consecutive rows hits 16 distinct bank groups; then each wave's query block [16 queries][8 float4].
// Per chunk a wave issues DT_XPW = 8 x pieces (8 rows × one line each) + 1 or 2 query pieces.
#ifndef HIPANN_DT_WAVES
#define HIPANN_DT_WAVES 8
#endif
#ifndef HIPANN_DT_NW
#define HIPANN_DT_NW 8
#endif
#ifndef HIPANN_DT_BK
#define HIPANN_DT_BK 32
#endif
#ifndef HIPANN_DT_BLOCKS
#define HIPANN_DT_BLOCKS 2
#endif
constexpr int DT_WAVES = HIPANN_DT_WAVES;
constexpr int DT_THREADS = 64 * DT_WAVES;
constexpr int DT_BLOCKS = HIPANN_DT_BLOCKS;         // resident blocks per CU (LDS and VGPR budget)
constexpr int DT_R = 4;
constexpr int DT_NW = HIPANN_DT_NW;
constexpr int DT_G = DT_WAVES * DT_NW;
#ifndef HIPANN_DT_QB
#define HIPANN_DT_QB 4
#endif
#ifndef HIPANN_DT_PF
#define HIPANN_DT_PF 0
#endif
constexpr int DT_QB = HIPANN_DT_QB;                 // queries per register block (q float4 live at once)
constexpr bool DT_PF = HIPANN_DT_PF;
#ifndef HIPANN_DT_EXPERIMENT
#define HIPANN_DT_EXPERIMENT 0  // tuning builds only: 1 = skip the FMAs, 2 = skip the row DMA (wrong results)
#endif                // L2 prefetch of the chunk after the one being DMA'd
constexpr int DT_TR = 64 * DT_R;
constexpr int DT_BK = HIPANN_DT_BK;
constexpr int DT_F4 = DT_BK / 4;                    // float4 per row per chunk
constexpr int DT_RP = 64 / DT_F4;                   // rows per x piece
constexpr int DT_SWZ = 16 / DT_F4;                  // rows sharing one swizzle value
constexpr int DT_XF4 = DT_TR * DT_F4;               // float4 of rows per stage
constexpr int DT_XPW = DT_XF4 / 64 / DT_WAVES;      // x pieces per wave per chunk
constexpr int DT_QF4 = (DT_NW * DT_F4 + 63) / 64 * 64;  // float4 of queries per wave per stage (whole pieces)
constexpr int DT_STAGE_F4 = DT_XF4 + DT_WAVES * DT_QF4;
constexpr int DT_STAGES = 2;
constexpr bool DT_DPP = false;  // q via DPP row_newbcast: measured 7% slower than LDS broadcast reads
static_assert(IVF_CH % DT_TR == 0, "row chunks are whole tiles");
static_assert(DT_XPW * 64 * DT_WAVES == DT_XF4 && DT_QF4 % 64 == 0 && DT_QF4 <= 128, "piece split");
static_assert((DT_F4 & (DT_F4 - 1)) == 0 && DT_F4 <= 16 && (DT_TR / DT_WAVES) % (DT_SWZ * DT_F4) == 0,
              "swizzle: a wave's rows start on a swizzle period");
static_assert(DT_STAGES * DT_STAGE_F4 * 16 * DT_BLOCKS <= 160 * 1024, "DT_BLOCKS blocks per CU");

typedef __attribute__((address_space(3))) void *ivf_lds_ptr;
typedef __attribute__((address_space(1))) void *ivf_gbl_ptr;

__device__ __forceinline__ void ivf_glds16(const float *src, float *lds_wave_base) {
    __builtin_amdgcn_global_load_lds((ivf_gbl_ptr)(src), (ivf_lds_ptr)(lds_wave_base), 16, 0, 0);
}

// Wait until at most N of this wave's DMA instructions are outstanding, then a raw barrier: past it
// every wave's pieces of the chunk to be read have landed and every wave has finished reading the
// stage the next issue overwrites.  "memory" pins LDS accesses around it.
template <int N>
__device__ __forceinline__ void ivf_dt_wait_barrier(float &pf, float (&xnv)[DT_R]) {
    static_assert(DT_R == 4, "operand list");
    asm volatile("s_waitcnt vmcnt(%5)\n\ts_barrier"
                 : "+v"(pf), "+v"(xnv[0]), "+v"(xnv[1]), "+v"(xnv[2]), "+v"(xnv[3])
                 : "n"(N)
                 : "memory");
}

// L2 prefetch: a dword load per 128-B line of the chunk after the one being DMA'd, into the sink
// register pf.  pf is read and written by every prefetch and by every wait, so it stays one live
// register for the whole loop (never reused while a prefetch into it is in flight); nothing reads
// its value.  The wait leaves the newest prefetch outstanding (vmcnt(1)).
__device__ __forceinline__ void ivf_prefetch_line(float &pf, const float *p) {
    asm volatile("global_load_dword %0, %1, off" : "+v"(pf) : "v"(p) : "memory");
}

// ‖x‖² of the lane's 4 rows of the tile being started, loaded behind the compiler's back (a plain
// load would make it wait vmcnt(0) — draining the DMA ring — at the first use): issued right after
// a barrier, ahead of that chunk's DMA and prefetch, so the next barrier's vmcnt(1) retires it long
// before the tile's epilogue reads it.  Rows past the chunk read any valid element (never offered).
__device__ __forceinline__ void ivf_load_norms(float (&xnv)[DT_R], const float *xn, int64_t t0, int64_t r1,
                                               int lane) {
#pragma unroll
    for (int r = 0; r < DT_R; ++r) {
        const int64_t row = t0 + lane + 64 * r < r1 ? t0 + lane + 64 * r : r1 - 1;
        asm volatile("global_load_dword %0, %1, off" : "=v"(xnv[r]) : "v"(xn + row) : "memory");
    }
}

// acc[r][J0 + j] += q_j · x_r over one float4 of dims, for the NB queries J0 .. J0 + NB − 1
// (q broadcast from LDS: one ds_read_b128 per query).
template <int NB, int J0, int NA>
__device__ __forceinline__ void ivf_dot_block(const float *__restrict__ Qw, int u, const float4 (&xv)[DT_R],
                                              float (&acc)[DT_R][NA]) {
    float4 qv[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) qv[j] = *reinterpret_cast<const float4 *>(Qw + ((J0 + j) * DT_F4 + u) * 4);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < DT_R; ++r) acc[r][J0 + j] = fmaf(qv[j].x, xv[r].x, acc[r][J0 + j]);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < DT_R; ++r) acc[r][J0 + j] = fmaf(qv[j].y, xv[r].y, acc[r][J0 + j]);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < DT_R; ++r) acc[r][J0 + j] = fmaf(qv[j].z, xv[r].z, acc[r][J0 + j]);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < DT_R; ++r) acc[r][J0 + j] = fmaf(qv[j].w, xv[r].w, acc[r][J0 + j]);
}

// acc += bcast16(q, lane N of each 16-lane row) · x — v_fmac_f32 with a DPP row_newbcast source.
// The backend does not fold v_mov_b32_dpp into v_fma_f32 (VOP3), so the VOP2 form is spelled out.
// q comes straight from a ds_read (no VALU write in front of the DPP read: no wait states needed).
template <int N>
__device__ __forceinline__ void ivf_fmac_bcast(float &acc, float q, float x) {
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(q), "v"(x), "n"(N));
}

template <int C>
__device__ __forceinline__ float ivf_comp(const float4 &v) {
    if constexpr (C == 0) return v.x;
    else if constexpr (C == 1) return v.y;
    else if constexpr (C == 2) return v.z;
    else return v.w;
}

// component C of one 4-dim step for queries J0 + Js (compile-time j for the DPP lane select)
template <int C, int J0, int NA, int NH, int... Js>
__device__ __forceinline__ void ivf_dpp_comp(std::integer_sequence<int, Js...>, const float (&V)[NH],
                                             const float4 (&xv)[DT_R], float (&acc)[DT_R][NA]) {
    (
        [&] {
#pragma unroll
            for (int r = 0; r < DT_R; ++r)
                ivf_fmac_bcast<4 * (Js & 3) + C>(acc[r][J0 + Js], V[Js >> 2], ivf_comp<C>(xv[r]));
        }(),
        ...);
}

// Same contract as ivf_dot_block, q values via DPP: lane m of each 16-lane row of V[h] holds
// q_{J0 + 4h + m/4}[4u + m%4], so a 4-dim step costs ⌈NB/4⌉ ds_read_b32 instead of NB ds_read_b128.
template <int NB, int J0, int NA>
__device__ __forceinline__ void ivf_dot_block_dpp(const float *__restrict__ Qw, int u, int lane,
                                                  const float4 (&xv)[DT_R], float (&acc)[DT_R][NA]) {
    constexpr int NH = (NB + 3) / 4;
    float V[NH];
    const int m = lane & 15;
#pragma unroll
    for (int h = 0; h < NH; ++h) V[h] = Qw[(J0 + 4 * h + (m >> 2)) * DT_BK + 4 * u + (m & 3)];
    using Seq = std::make_integer_sequence<int, NB>;
    ivf_dpp_comp<0, J0, NA, NH>(Seq{}, V, xv, acc);
    ivf_dpp_comp<1, J0, NA, NH>(Seq{}, V, xv, acc);
    ivf_dpp_comp<2, J0, NA, NH>(Seq{}, V, xv, acc);
    ivf_dpp_comp<3, J0, NA, NH>(Seq{}, V, xv, acc);
}

// all NW queries of the wave, in register blocks of ≤ DT_QB
template <int NW, int J0, int NA>
__device__ __forceinline__ void ivf_dot_blocks(const float *__restrict__ Qw, int u, int lane, const float4 (&xv)[DT_R],
                                               float (&acc)[DT_R][NA]) {
    if constexpr (NW - J0 > 0) {
        constexpr int NB = NW - J0 < DT_QB ? NW - J0 : DT_QB;
        if constexpr (DT_DPP) ivf_dot_block_dpp<NB, J0, NA>(Qw, u, lane, xv, acc);
        else ivf_dot_block<NB, J0, NA>(Qw, u, xv, acc);
        ivf_dot_blocks<NW, J0 + NB, NA>(Qw, u, lane, xv, acc);
    }
}

template <int NW, bool IP>
__device__ __forceinline__ void ivf_dot_item(int d, const float *__restrict__ codes, const float *__restrict__ xn,
                                             int64_t r0, int64_t r1, const float *qsrc0, const float *qsrc1,
                                             const float *qn, int wq0, const int *__restrict__ bucket, int boff,
                                             int nprobe, const int *__restrict__ slot_off, int chunk, int k,
                                             float *ring, float *__restrict__ part_d, int *__restrict__ part_i) {
    constexpr int NA = NW > 0 ? NW : 1;
    constexpr int QP = NW * DT_F4 > 64 ? 2 : 1;  // query pieces per chunk
    constexpr int PIECES = DT_XPW + QP;          // DMA instructions per wave per chunk
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nk = (d + DT_BK - 1) / DT_BK;
    const int ntile = (int)((r1 - r0 + DT_TR - 1) / DT_TR);
    const int total = ntile * nk;

    // ---- issue side: x piece i of wave w = rows w·(TR/WAVES) + i·RP + lane / F4; the lane's float4
    // slot (lane % F4) of its row holds logical float4 (lane % F4) ^ swz(row) ----
    const int prow = wave * (DT_TR / DT_WAVES) + lane / DT_F4;
    // (recomputed per issue: registers are the scarce resource here)
    auto xc4 = [&](int i) { return 4 * ((lane % DT_F4) ^ (((i * DT_RP + lane / DT_F4) / DT_SWZ) & (DT_F4 - 1))); };
    const int qc4 = 4 * (lane % DT_F4);
    int it_kc = 0, it_buf = 0;
    int64_t it_t0 = r0;
    float pf = 0.f, xnv[DT_R] = {0.f, 0.f, 0.f, 0.f};
    static_assert(!DT_PF || (DT_STAGES == 2 && DT_TR / DT_WAVES == 32), "one prefetch dword per wave lane pair per chunk");
    auto issue = [&]() {
        float *stage = ring + (size_t)it_buf * DT_STAGE_F4 * 4;
        const int k0 = it_kc * DT_BK;
        const bool full_k = k0 + DT_BK <= d;
        if (HIPANN_DT_EXPERIMENT == 2) {
        } else if (it_t0 + DT_TR <= r1 && full_k) {  // interior tile, whole chunk: no clamps
            const float *base = codes + (it_t0 + prow) * (int64_t)d + k0;
#pragma unroll
            for (int i = 0; i < DT_XPW; ++i)
                ivf_glds16(base + (int64_t)(DT_RP * i) * d + xc4(i), stage + (size_t)(wave * DT_XPW + i) * 64 * 4);
        } else {  // rows past the chunk re-load its last row, dims past d any valid float4 (never read)
#pragma unroll
            for (int i = 0; i < DT_XPW; ++i) {
                const int64_t row = it_t0 + prow + DT_RP * i < r1 ? it_t0 + prow + DT_RP * i : r1 - 1;
                const int kk = k0 + xc4(i) < d ? k0 + xc4(i) : d - 4;
                ivf_glds16(codes + row * (int64_t)d + kk, stage + (size_t)(wave * DT_XPW + i) * 64 * 4);
            }
        }
        const int kq = k0 + qc4 < d ? k0 + qc4 : d - 4;
        float *qdst = stage + (size_t)(DT_XF4 + wave * DT_QF4) * 4;
        ivf_glds16(qsrc0 + kq, qdst);
        if (QP == 2) ivf_glds16(qsrc1 + kq, qdst + 64 * 4);
        if (++it_kc == nk) { it_kc = 0; it_t0 += DT_TR; }
        it_buf = it_buf == DT_STAGES - 1 ? 0 : it_buf + 1;
        // warm L2 with the next chunk's lines: rows wave·(TR/WAVES) + (lane % 32), one dword per line
        if constexpr (DT_PF) {
            const int64_t prow_pf = it_t0 + wave * (DT_TR / DT_WAVES) + (lane & 31);
            const int64_t row = prow_pf < r1 ? prow_pf : r1 - 1;
            ivf_prefetch_line(pf, codes + row * (int64_t)d + it_kc * DT_BK);
        }
    };

    // ---- compute side ----
    WaveList<1, int> lists[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) lists[j].init();
    // ‖q_j‖² held by lane j (read back with readlane in the epilogue: no per-query SGPRs)
    const float qn_lane = (!IP && lane < NW) ? qn[bucket[boff + wq0 + lane] / nprobe] : 0.f;
    float acc[DT_R][NA];
#pragma unroll
    for (int r = 0; r < DT_R; ++r)
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[r][j] = 0.f;

    const int swz = (lane / DT_SWZ) & (DT_F4 - 1);  // swz(row) of rows lane + 64r
#pragma unroll
    for (int s = 0; s < DT_STAGES - 1; ++s)
        if (s < total) issue();
    int kc = 0, buf = 0;
    int64_t t0 = r0;
    for (int c = 0; c < total; ++c) {
        // chunk c's pieces (and any norms issued before them) landed; the prefetch issued after
        // them may stay in flight
        ivf_dt_wait_barrier<DT_PF ? 1 : 0>(pf, xnv);
        if (!IP && NW > 0 && kc == 0) ivf_load_norms(xnv, xn, t0, r1, lane);
        if (c + DT_STAGES - 1 < total) issue();
        const float *X = ring + (size_t)buf * DT_STAGE_F4 * 4;
        const float *Qw = X + (size_t)(DT_XF4 + wave * DT_QF4) * 4;
        const int k0 = kc * DT_BK;
        const int nu = d - k0 >= DT_BK ? DT_F4 : (d - k0) / 4;
        if (NW > 0) {
#pragma unroll 1
            for (int u = 0; u < nu; ++u) {
                float4 xv[DT_R];
                const float *xl = X + (lane * DT_F4 + (u ^ swz)) * 4;
#pragma unroll
                for (int r = 0; r < DT_R; ++r) xv[r] = *reinterpret_cast<const float4 *>(xl + r * 64 * DT_F4 * 4);
                if (HIPANN_DT_EXPERIMENT != 1) ivf_dot_blocks<NW, 0, NA>(Qw, u, lane, xv, acc);
                else acc[0][0] += xv[0].x + xv[1].y + xv[2].z + xv[3].w;
            }
        }
        if (++kc == nk) {  // tile done: offer its rows
            if (NW > 0) {
                if (nk == 1)  // the norms were issued in this very chunk: no barrier has retired them yet
                    asm volatile("s_waitcnt vmcnt(0)"
                                 : "+v"(pf), "+v"(xnv[0]), "+v"(xnv[1]), "+v"(xnv[2]), "+v"(xnv[3])::"memory");
#pragma unroll
                for (int r = 0; r < DT_R; ++r) {
                    const int64_t row = t0 + lane + 64 * r;
                    const bool v = row < r1;
                    const float xnr = xnv[r];
#pragma unroll
                    for (int j = 0; j < NW; ++j) {
                        float key;
                        if (IP) {
                            key = -acc[r][j];
                        } else {
                            const float qnj = __builtin_bit_cast(
                                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, qn_lane), j));
                            key = fmaf(-2.f, acc[r][j], qnj + xnr);
                            key = key < 0.f ? 0.f : key;
                        }
                        lists[j].template offer<false>(v ? key : __builtin_inff(), v ? (int)row : 0x7fffffff, k - 1);
                        acc[r][j] = 0.f;
                    }
                }
            }
            kc = 0;
            t0 += DT_TR;
        }
        buf = buf == DT_STAGES - 1 ? 0 : buf + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(pf)::"memory");  // retire the last prefetch before pf dies
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const int pr = bucket[boff + wq0 + j];
        const int64_t off = (int64_t)(slot_off[pr] + chunk) * k;
        lists[j].store(part_d + off, part_i + off, k);
    }
}

// nwq (wave-uniform) → ivf_dot_item<nwq>
template <int N, bool IP>
__device__ __forceinline__ void ivf_dot_dispatch(int nwq, int d, const float *codes, const float *xn, int64_t r0,
                                                 int64_t r1, const float *qsrc0, const float *qsrc1, const float *qn,
                                                 int wq0, const int *bucket, int boff, int nprobe, const int *slot_off,
                                                 int chunk, int k, float *ring, float *part_d, int *part_i) {
    if constexpr (N >= DT_NW) {
        ivf_dot_item<DT_NW, IP>(d, codes, xn, r0, r1, qsrc0, qsrc1, qn, wq0, bucket, boff, nprobe, slot_off, chunk, k,
                                ring, part_d, part_i);
    } else {
        if (nwq == N)
            ivf_dot_item<N, IP>(d, codes, xn, r0, r1, qsrc0, qsrc1, qn, wq0, bucket, boff, nprobe, slot_off, chunk, k,
                                ring, part_d, part_i);
        else
            ivf_dot_dispatch<N + 1, IP>(nwq, d, codes, xn, r0, r1, qsrc0, qsrc1, qn, wq0, bucket, boff, nprobe,
                                        slot_off, chunk, k, ring, part_d, part_i);
    }
}

template <bool IP>
__global__ void __launch_bounds__(DT_THREADS, DT_BLOCKS * DT_THREADS / 256)
ivf_scan_dot(const float *__restrict__ Q, const float *__restrict__ qn, int d, const float *__restrict__ codes,
             const float *__restrict__ xn, const int64_t *__restrict__ list_off, const int *__restrict__ list_len, const int *__restrict__ cnt,
             const int *__restrict__ bucket_off, const int *__restrict__ item_off, const int *__restrict__ bucket,
             const int *__restrict__ slot_off, int nlist, int nprobe, int k, float *__restrict__ part_d,
             int *__restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float ring[];
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
    const int ng = (c + DT_G - 1) / DT_G;
    const int rem = item - item_off[l];
    const int chunk = rem / ng, g = rem - chunk * ng;  // (row chunk, query group), group fastest
    const int q_begin = (int)((int64_t)g * c / ng), q_end = (int)((int64_t)(g + 1) * c / ng);
    const int nqi = q_end - q_begin;
    const int64_t r0 = lr0 + (int64_t)chunk * IVF_CH;
    const int64_t r1 = r0 + IVF_CH < lr1 ? r0 + IVF_CH : lr1;
    const int boff = bucket_off[l] + q_begin;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wq0 = __builtin_amdgcn_readfirstlane(wave * nqi / DT_WAVES);
    const int nwq = __builtin_amdgcn_readfirstlane((wave + 1) * nqi / DT_WAVES - wave * nqi / DT_WAVES);
    // query-piece lanes: piece h, lane → slot (64h + lane) / DT_F4 of this wave's block (slots past nwq
    // re-load the wave's first query)
    const int s0 = lane / DT_F4, s1 = (64 + lane) / DT_F4;
    const float *qsrc0 = Q + (int64_t)(bucket[boff + wq0 + (s0 < nwq ? s0 : 0)] / nprobe) * d;
    const float *qsrc1 = Q + (int64_t)(bucket[boff + wq0 + (s1 < nwq ? s1 : 0)] / nprobe) * d;
ivf_dot_dispatch<0, IP>(nwq, d, codes, xn, r0, r1, qsrc0, qsrc1, qn, wq0, bucket, boff, nprobe, slot_off, chunk, k,
                           ring, part_d, part_i);
}

// Merge each query's partial lists (its contiguous slot range), mapping shard-local rows to labels.
template <int S>
__global__ void __launch_bounds__(256)
ivf_merge_topk(const float *__restrict__ pd, const int *__restrict__ pi, const int64_t *__restrict__ ids,
               int64_t nrows, const int *__restrict__ slot_off, int nprobe, int64_t nq, int k, int kout, float out_sign,
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
            if (raw >= 0 && raw < nrows && !(v == __builtin_inff())) {  // pads: 0x7fffffff >= nrows
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
// ivf_scan_slot_bigk — the k > 64 path (faiss-metal's select handles k ≤ 2048, MetalSelect.mm:31-74).
// One block per partial-list slot (pair q·nprobe + p, row chunk c of the probed list): the query in
// LDS, every chunk row's direct-form key (FAISS IVFFlatScanner: Σ(q−x)², or −q·x) computed by one
// wave per row, then the ≤ 2048 (key, row) pairs bitonic-sorted in LDS and the first k written.
// Query-major (each list is re-read per probing query): a correctness path for large k, not the
// throughput path.
// ---------------------------------------------------------------------------------------------
template <bool IP>
__global__ void __launch_bounds__(256)
ivf_scan_slot_bigk(const float *__restrict__ Q, int d, const float *__restrict__ codes,
                   const int64_t *__restrict__ list_off, const int *__restrict__ list_len, const int64_t *__restrict__ probes, int64_t npairs,
                   int nprobe, const int *__restrict__ slot_off, int k, float *__restrict__ part_d,
                   int *__restrict__ part_i) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *sk = sm;                                          // [IVF_CH] keys
    int *si = reinterpret_cast<int *>(sm + IVF_CH);          // [IVF_CH] rows
    float *qv = sm + 2 * IVF_CH;                             // [d] query
    const int slot = blockIdx.x;
    if (slot >= slot_off[npairs]) return;  // the grid is sized for the worst case
    // pair owning this slot: the last i with slot_off[i] <= slot (pairs with no slots are skipped)
    int64_t lo = 0, hi = npairs - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (slot_off[mid] <= slot) lo = mid; else hi = mid - 1;
    }
    const int64_t pair = lo;
    const int chunk = slot - slot_off[pair];
    const int64_t l = probes[pair];
    const int64_t lend = list_off[l] + list_len[l];
    const int64_t r0 = list_off[l] + (int64_t)chunk * IVF_CH;
    const int64_t r1 = r0 + IVF_CH < lend ? r0 + IVF_CH : lend;
    const int len = (int)(r1 - r0);
    const float *q = Q + (pair / nprobe) * (int64_t)d;
    for (int j = threadIdx.x; j < d; j += 256) qv[j] = q[j];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int r = wave; r < IVF_CH; r += 4) {
        float acc = 0.f;
        if (r < len) {
            const float *x = codes + (r0 + r) * (int64_t)d;
            for (int j = lane; j < d; j += 64) {
                if (IP) acc = fmaf(qv[j], x[j], acc);
                else { const float t = qv[j] - x[j]; acc = fmaf(t, t, acc); }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        }
        if (lane == 0) {
            sk[r] = r < len ? (IP ? -acc : acc) : __builtin_inff();
            si[r] = r < len ? (int)(r0 + r) : 0x7fffffff;
        }
    }
    __syncthreads();
    // bitonic sort of IVF_CH pairs, ascending (key, row)
    for (int size = 2; size <= IVF_CH; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < IVF_CH / 2; t += 256) {
                const int a = 2 * t - (t & (stride - 1)), b = a + stride;
                const bool up = (a & size) == 0;
                const float ka = sk[a], kb = sk[b];
                const int ia = si[a], ib = si[b];
                const bool b_less = kb < ka || (kb == ka && ib < ia);
                if (b_less == up) { sk[a] = kb; sk[b] = ka; si[a] = ib; si[b] = ia; }
            }
            __syncthreads();
        }
    }
    const int64_t off = (int64_t)slot * k;
    for (int e = threadIdx.x; e < k; e += 256) {
        part_d[off + e] = e < IVF_CH ? sk[e] : __builtin_inff();
        part_i[off + e] = e < IVF_CH ? si[e] : 0x7fffffff;
    }
}

void launch_ivf_scan_bigk(const float *Q, int d, int metric, const float *codes, const int64_t *list_off,
                          const int *list_len, const int64_t *probes, int64_t npairs, int nprobe, const int *slot_off, int64_t nslots,
                          int k, float *pd, int *pi, hipStream_t st) {
    if (nslots <= 0) return;
    HIPANN_REQUIRE(nslots < (int64_t)0x7fffffff, "too many slots");
    const size_t smem = (size_t)2 * IVF_CH * 4 + (size_t)d * 4;
    HIPANN_REQUIRE(smem <= 64 * 1024, "dimension too large for the k > 64 IVF path");
    dim3 grid((unsigned)nslots), block(256);
    if (metric == kIP)
        hipLaunchKernelGGL(ivf_scan_slot_bigk<true>, grid, block, smem, st, Q, d, codes, list_off, list_len, probes, npairs,
                           nprobe, slot_off, k, pd, pi);
    else
        hipLaunchKernelGGL(ivf_scan_slot_bigk<false>, grid, block, smem, st, Q, d, codes, list_off, list_len, probes, npairs,
                           nprobe, slot_off, k, pd, pi);
    HIPANN_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// HIPANN_IVF_PLAN_SPLIT=1: the list-major count / plan / slot scan / fill sequence (A/B)
bool ivf_plan_query_major() {
    static const bool split = [] { const char *e = std::getenv("HIPANN_IVF_PLAN_SPLIT"); return e && std::atoi(e); }();
    return !split;
}

void launch_ivf_plan(const int64_t *probes, int64_t nq, int nprobe, const int *list_len, int nlist, int group,
                     int *cnt, int *bucket_off, int *item_off, int *cursor, int *bucket, int *slot_off,
                     hipStream_t st, int *nflag_reset, unsigned *qbound, int *ccnt, int *qtot, bool counted,
                     int *ccnt_next, int *cursor_next) {
    const int64_t npairs = nq * nprobe;
    if (ivf_plan_query_major() && ccnt && qtot) {
        const unsigned gq = (unsigned)std::max<int64_t>(1, ceil_div(nq, (int64_t)4));
        if (nq > 0 && !counted)  // counted: the coarse probe select already did this step (IvfPlanHook)
            hipLaunchKernelGGL(ivf_count_q, dim3(gq), dim3(256), 0, st, probes, nq, nprobe, list_len, nlist, ccnt,
                               slot_off, qtot);
        // one launch (double-buffered counts and cursors) when the lists fit the block's LDS; HIPANN_IVF_PLANFILL=0
        // keeps the two (A/B)
        static const bool fused_env = [] { const char *e = std::getenv("HIPANN_IVF_PLANFILL"); return !e || std::atoi(e); }();
        if (fused_env && ccnt_next && cursor_next && nlist <= kPlanFillMaxList && nq > 0) {
            hipLaunchKernelGGL(ivf_planfill_q, dim3(gq), dim3(256), 0, st, probes, nq, nprobe, list_len, nlist, group,
                               ccnt, ccnt_next, cursor, cursor_next, qtot, slot_off, npairs, cnt, bucket_off, item_off,
                               bucket, nflag_reset, qbound);
            HIPANN_CHECK(hipGetLastError());
            return;
        }
        hipLaunchKernelGGL(ivf_plan_q, dim3(1), dim3(1024), 0, st, ccnt, list_len, nlist, group, cnt, bucket_off,
                           item_off, cursor, qtot, nq, npairs, slot_off, nflag_reset, qbound);
        if (nq > 0)
            hipLaunchKernelGGL(ivf_fill_q, dim3(gq), dim3(256), 0, st, probes, nq, nprobe, list_len, nlist, qtot,
                               bucket_off, cursor, bucket, slot_off);
        if (cursor_next)  // the fused path expects the other parity's cursors at zero
            HIPANN_CHECK(hipMemsetAsync(cursor_next, 0, sizeof(int) * kPlanCopies * (size_t)nlist, st));
        HIPANN_CHECK(hipGetLastError());
        return;
    }
    if (nflag_reset) HIPANN_CHECK(hipMemsetAsync(nflag_reset, 0, sizeof(int), st));
    if (qbound) HIPANN_CHECK(hipMemsetD32Async((hipDeviceptr_t)qbound, 0xff800000, (size_t)nq, st));
    HIPANN_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)nlist, st));
    if (npairs > 0)
        hipLaunchKernelGGL(ivf_count, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, st, probes, npairs, list_len,
                           nlist, cnt);
    hipLaunchKernelGGL(ivf_plan, dim3(1), dim3(1024), 0, st, cnt, list_len, nlist, group, bucket_off, item_off,
                       cursor);
    hipLaunchKernelGGL(ivf_slot_scan, dim3(1), dim3(1024), 0, st, probes, npairs, list_len, nlist, slot_off);
    if (npairs > 0)
        hipLaunchKernelGGL(ivf_fill, dim3((unsigned)ceil_div(npairs, 256)), dim3(256), 0, st, probes, npairs, list_len,
                           nlist, bucket_off, cursor, bucket);
    HIPANN_CHECK(hipGetLastError());
}

// Upper bound on work items given the largest list's chunk count.
// Σ_l ceil(cnt_l/G)·nch_l ≤ Σ_l (cnt_l/G + 1)·nch_l ≤ ceil(npairs/G)·max_nch + Σ_l nch_l.
int64_t ivf_max_items(int64_t nq, int nprobe, int nlist, int max_nch, int64_t nrows, int group) {
    const int64_t npairs = nq * nprobe;  // (a wide group size only lowers the count)
    return ceil_div(npairs, (int64_t)ivf_group_min(group)) * std::max(max_nch, 1) + ceil_div(nrows, IVF_CH) + nlist;
}

int ivf_mfma_group(int d);            // ivf_mfma.hip
int ivf_mfma_bf_group(int d, int np);  // ivf_mfma.hip

int ivf_group_size(int form, int d) {
    if (ivf_form_split(form)) return ivf_mfma_bf_group(d, ivf_form_terms(form));
    return form == kFormDecomposed ? ivf_mfma_group(d) : form == kFormDecomposedValu ? DT_G : IVF_G;
}

int ivf_chunk_rows() { return IVF_CH; }

size_t ivf_scan_smem_bytes() { return (size_t)2 * (IVF_TR + IVF_G) * IVF_LD * sizeof(float); }
static size_t ivf_scan_dot_smem_bytes() { return (size_t)DT_STAGES * DT_STAGE_F4 * 16; }

bool ivf_dot_supported(const float *Q, int d, const float *codes) {
    return (d % 4 == 0) && ((uintptr_t)Q % 16 == 0) && ((uintptr_t)codes % 16 == 0);
}

void launch_ivf_scan(const float *Q, const float *qn, int d, int metric, int form, const float *codes,
                     const float *xn, const int64_t *list_off, const int *list_len, const int *cnt,
                     const int *bucket_off, const int *item_off, const int *bucket, const int *slot_off, int nlist,
                     int nprobe, int64_t nq,
                     int k, int64_t max_items, unsigned *qbound, float *pd, int *pi, hipStream_t st) {
    if (max_items <= 0) return;
    HIPANN_REQUIRE(max_items < (int64_t)0x7fffffff, "too many IVF work items");
    HIPANN_REQUIRE(form != kFormDecomposed, "the MFMA scan is launched with its tiled codes (launch_ivf_scan_mfma)");
    if (form == kFormDecomposedValu) {
        HIPANN_REQUIRE(ivf_dot_supported(Q, d, codes), "decomposed IVF scan needs d % 4 == 0 and 16-B aligned data");
        HIPANN_REQUIRE(metric == kIP || (qn && xn), "decomposed L2 scan needs query and row norms");
        dim3 grid((unsigned)max_items), block(DT_THREADS);
        const size_t smem = ivf_scan_dot_smem_bytes();
#define HIPANN_DOT_ARGS Q, qn, d, codes, xn, list_off, list_len, cnt, bucket_off, item_off, bucket, slot_off, nlist, nprobe, k, pd, pi
        if (metric == kIP) hipLaunchKernelGGL((ivf_scan_dot<true>), grid, block, smem, st, HIPANN_DOT_ARGS);
        else hipLaunchKernelGGL((ivf_scan_dot<false>), grid, block, smem, st, HIPANN_DOT_ARGS);
#undef HIPANN_DOT_ARGS
    } else {
        const bool vec4 = ivf_dot_supported(Q, d, codes);
        dim3 grid((unsigned)max_items), block(IVF_THREADS);
        const size_t smem = ivf_scan_smem_bytes();
#define HIPANN_IVF_ARGS Q, d, codes, list_off, list_len, cnt, bucket_off, item_off, bucket, slot_off, nlist, nprobe, nq, k, pd, pi
        if (vec4) {
            if (metric == kIP) hipLaunchKernelGGL((ivf_scan_topk<true, true>), grid, block, smem, st, HIPANN_IVF_ARGS);
            else hipLaunchKernelGGL((ivf_scan_topk<true, false>), grid, block, smem, st, HIPANN_IVF_ARGS);
        } else {
            if (metric == kIP) hipLaunchKernelGGL((ivf_scan_topk<false, true>), grid, block, smem, st, HIPANN_IVF_ARGS);
            else hipLaunchKernelGGL((ivf_scan_topk<false, false>), grid, block, smem, st, HIPANN_IVF_ARGS);
        }
#undef HIPANN_IVF_ARGS
    }
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_merge(const float *pd, const int *pi, const int64_t *ids, int64_t nrows, const int *slot_off, int nprobe, int64_t nq,
                      int k, int kout, float out_sign, float *D, int64_t *I, hipStream_t st) {
    if (nq <= 0) return;
    dim3 grid((unsigned)ceil_div(nq, 4)), block(256);
    const int S = (kout + 63) / 64;
#define HIPANN_IVF_MERGE(s)                                                                                           \
    if (S <= s) {                                                                                                     \
        hipLaunchKernelGGL(ivf_merge_topk<s>, grid, block, 0, st, pd, pi, ids, nrows, slot_off, nprobe, nq, k, kout, \
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

namespace hipann {

// Direct-form sums of 4 rows against one query, lane-strided over the dims (e = lane, lane + 64, ...):
// the loads of 4 strides are issued before their fmas (3 memory round trips at d = 768 instead of 12);
// every accumulator still adds its terms in e order, so the sums are the one-stride loop's bit for bit.
template <bool IP>
__device__ __forceinline__ void rerank_rows4(const float *__restrict__ qp, const float *const (&xr)[4], int d, int lane,
                                             float (&acc)[4]) {
    int e = lane;
    for (; e + 192 < d; e += 256) {
        float qv[4], xv[4][4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qv[s] = qp[e + 64 * s];
#pragma unroll
            for (int u = 0; u < 4; ++u) xv[s][u] = xr[u][e + 64 * s];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (IP) acc[u] = fmaf(qv[s], xv[s][u], acc[u]);
                else {
                    const float t = qv[s] - xv[s][u];
                    acc[u] = fmaf(t, t, acc[u]);
                }
            }
    }
    for (; e < d; e += 64) {
        const float qv = qp[e];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float xv = xr[u][e];
            if (IP) acc[u] = fmaf(qv, xv, acc[u]);
            else {
                const float t = qv - xv;
                acc[u] = fmaf(t, t, acc[u]);
            }
        }
    }
}

#ifndef HIPANN_RR_OLDSEL
#define HIPANN_RR_OLDSEL 0  // A/B builds: the 32-barrier block select instead of rerank_wave_select
#endif
#ifndef HIPANN_RR_PROF
#define HIPANN_RR_PROF 0  // tuning builds: wave 0's per-phase shader clocks of the wide rerank, summed in rr_prof
#endif
#ifndef HIPANN_RR_STAMP
#define HIPANN_RR_STAMP 0  // tuning builds: per-query wall-clock stamps (100 MHz) of the wide rerank's phases
#endif
#if HIPANN_RR_STAMP
__device__ long long rr_stamp[4096 * 8];
#define RR_STAMP_Q(qq, i) do { if (threadIdx.x == 0 && (qq) < 4096) rr_stamp[(qq) * 8 + (i)] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
#define RR_STAMP(i) RR_STAMP_Q(q, i)
#else
#define RR_STAMP(i) do { } while (0)
#define RR_STAMP_Q(qq, i) do { } while (0)
#endif
#if HIPANN_RR_PROF
__device__ unsigned long long rr_prof[16];
#define RR_MARK(i) do { if (wv == 0) { const long long t_ = clock64(); if (lane == 0) atomicAdd(&rr_prof[i], (unsigned long long)(t_ - rr_t)); rr_t = t_; } } while (0)
#else
#define RR_MARK(i) do { } while (0)
#endif
#if HIPANN_RR_PROF
#define RR_COUNT(i) do { if (wv == 0 && lane == 0) atomicAdd(&rr_prof[i], 1ull); } while (0)
#else
#define RR_COUNT(i) do { } while (0)
#endif
// HIPANN_RERANK_LISTS=1: the rerank merges with per-wave lists only (A/B of rerank_block_select).
__device__ __forceinline__ bool rerank_lists() {
#ifdef HIPANN_RERANK_LISTS
    return true;
#else
    return false;
#endif
}

// The k best scan keys of a query's ≤ 64·WV·J candidates (pd/pi: keys and row ids, contiguous) by one
// bitwise select over the whole block: candidate c = (j·WV + wave)·64 + lane sits in register j as an
// order-preserving u32 (pads, rows out of range, +inf and NaN keys excluded — the entries the list merge
// never admits); 32 steps find the k-th smallest value T (per step J ballots + popcounts per wave and
// one barrier for the block sum), the keys < T and then the first keys == T (in (wave, j, lane) order)
// are compacted into LDS, and wave 0 sorts them into L (lanes < k: ascending (key, row); pads past the
// candidates).  A tie at T may pick different rows than the (key, row) lists would — harmless: every
// row left out still has scan key ≥ K_k, which is all the bound check assumes.
// bound (the scan's final per-query bound, an upper bound of the k-th smallest key): when at most 64 candidates
// have key <= bound — the usual case: the lists' early entries were admitted under looser running bounds —
// they are compacted and sorted directly (the k smallest (key, row) among them are the k smallest overall), no
// 32-step search.
template <int WV, int J>
__device__ __forceinline__ void rerank_block_select(const float *__restrict__ pd, const int *__restrict__ pi,
                                                    int64_t total, int k, int64_t nrows, float *sd, int *si,
                                                    int (*scnt)[WV], WaveList<1, int> &L,
                                                    float bound, long long &rr_t) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    (void)rr_t;
    float v[J];
    int r[J];
    unsigned u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t c = ((int64_t)j * WV + wv) * 64 + lane;
        v[j] = c < total ? pd[c] : __builtin_inff();
        r[j] = c < total ? pi[c] : -1;
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool ok = r[j] >= 0 && r[j] < nrows && v[j] == v[j] && !(v[j] == __builtin_inff());
        const float f = v[j] == 0.f ? 0.f : v[j];
        const unsigned b = __float_as_uint(f);
        u[j] = ok ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
    }
    RR_MARK(1);  // candidate loads
    if (bound < __builtin_inff()) {
        const unsigned long long lt = (1ull << lane) - 1ull;
        int nb = 0;
#pragma unroll
        for (int j = 0; j < J; ++j) nb += __popcll(__ballot(u[j] != 0xffffffffu && v[j] <= bound));
        if (lane == 0) scnt[0][wv] = nb;
        __syncthreads();
        int tot = 0, off = 0;
#pragma unroll
        for (int w = 0; w < WV; ++w) {
            tot += scnt[0][w];
            off += w < wv ? scnt[0][w] : 0;
        }
        RR_MARK(5);  // bound count + barrier
        if (tot <= 64) {  // block-uniform
            RR_COUNT(6);
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const bool a = u[j] != 0xffffffffu && v[j] <= bound;
                const unsigned long long ma = __ballot(a);
                if (a) { const int p = off + __popcll(ma & lt); sd[p] = v[j]; si[p] = r[j]; }
                off += __popcll(ma);
            }
            __syncthreads();
            if (wv == 0) {
                float kk = lane < tot ? sd[lane] : __builtin_inff();
                int cc = lane < tot ? si[lane] : IdTraits<int>::pad();
                wave_sort(kk, cc);
                L.d[0] = lane < k ? kk : __builtin_inff();
                L.id[0] = lane < k ? cc : IdTraits<int>::pad();
            }
            RR_MARK(2);  // compaction + sort
            return;
        }
        __syncthreads();  // every wave has read scnt before the search reuses it
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
        int tot = 0;
#pragma unroll
        for (int w = 0; w < WV; ++w) tot += scnt[par][w];
        if (tot < k) T = cand;
    }
    // compaction: this wave's counts below / at T, the waves' offsets through LDS
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
    int olt = 0, oeq = 0, tlt = 0;
#pragma unroll
    for (int w = 0; w < WV; ++w) {
        olt += w < wv ? scnt[0][w] : 0;
        oeq += w < wv ? scnt[1][w] : 0;
        tlt += scnt[0][w];
    }
    int plt = olt, peq = tlt + oeq;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool a = u[j] < T, b = u[j] == T && u[j] != 0xffffffffu;
        const unsigned long long ma = __ballot(a), mb = __ballot(b);
        if (a) { const int p = plt + __popcll(ma & lt); sd[p] = v[j]; si[p] = r[j]; }
        if (b) { const int p = peq + __popcll(mb & lt); if (p < k) { sd[p] = v[j]; si[p] = r[j]; } }
        plt += __popcll(ma);
        peq += __popcll(mb);
    }
    int tot_eq = 0;
#pragma unroll
    for (int w = 0; w < WV; ++w) tot_eq += scnt[1][w];
    const int nsel = tlt + tot_eq < k ? tlt + tot_eq : k;
    __syncthreads();
    if (wv == 0) {
        float kk = lane < nsel ? sd[lane] : __builtin_inff();
        int cc = lane < nsel ? si[lane] : IdTraits<int>::pad();
        wave_sort(kk, cc);
        L.d[0] = kk;
        L.id[0] = cc;
    }
    RR_MARK(2);  // 32-step search + compaction + sort
}


// The k best scan keys of a query's ≤ 64·WV·J candidates with ONE block barrier (rerank_block_select needs 32):
//   1. each wave loads its candidates (key, row) (c = (j·WV + wave)·64 + lane) in one round trip;
//   2. compacts the keys ≤ bound (finite, row in range) into its own LDS run in (j, lane) order, then finds its
//      run's k best by
//      a wave-local bitwise search (32 steps of ⌈m/64⌉ ballots, no barrier) — the bound (the scan's final
//      per-query bound) usually leaves a few dozen per wave;
//   3. after the barrier wave 0 takes the ≤ WV·k survivors, selects the k best the same way and sorts them by
//      (key, row) (wave_rank_sort).
// Ties at the k-th key keep the first in (wave, position) order — any choice is harmless: every row left out
// still has scan key ≥ K_k, all the bound check assumes.
template <int J>
__device__ __forceinline__ unsigned rws_kth_bits(const float *__restrict__ mk, int m, int k, unsigned &n_lt_out) {
    const int lane = threadIdx.x & 63;
    const int nj = (m + 63) >> 6;
    unsigned u[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * 64 + lane;
        float f = j < nj && e < m ? mk[e] : __builtin_inff();
        f = f == 0.f ? 0.f : f;
        const unsigned b = __float_as_uint(f);
        u[j] = j < nj && e < m ? ((b >> 31) ? ~b : (b | 0x80000000u)) : 0xffffffffu;
    }
    unsigned T = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = T | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < J; ++j)
            if (j < nj) cnt += __popcll(__ballot(u[j] < cand));
        if (cnt < k) T = cand;
    }
    (void)n_lt_out;
    return T;
}
__device__ __forceinline__ unsigned rws_bits(float f) {
    f = f == 0.f ? 0.f : f;
    const unsigned b = __float_as_uint(f);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}
// Copy the ≤ k best of run (mk, mp)[0, m) — keys < T, then the first keys == T — to (ok, op); returns the count.
template <int J>
__device__ __forceinline__ int rws_take(const float *__restrict__ mk, const int *__restrict__ mp, int m, int k, unsigned T,
                                        float *__restrict__ ok, int *__restrict__ op) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int nj = (m + 63) >> 6;
    int base = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * 64 + lane;
        const bool a = j < nj && e < m && rws_bits(mk[e]) < T;
        const unsigned long long ma = __ballot(a);
        if (a) { const int p = base + __popcll(ma & lt); ok[p] = mk[e]; op[p] = mp[e]; }
        base += __popcll(ma);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * 64 + lane;
        const bool b = j < nj && e < m && rws_bits(mk[e]) == T;
        const unsigned long long mb = __ballot(b);
        if (b) { const int p = base + __popcll(mb & lt); if (p < k) { ok[p] = mk[e]; op[p] = mp[e]; } }
        base += __popcll(mb);
    }
    return base < k ? base : k;
}
// The k best of a wave's run (mk, mp)[0, m) for m > 64 by narrowing (as flat_keys_kth): T_hi = the k-th smallest of
// the 64 lanes' minima (at least k entries lie at or below it), the entries ≤ T_hi compacted in (register, lane) order
// into (tk, tp), then the exact k-th and the take over that list of ≤ 64 — the same k entries as the bisection over
// the whole run (ties at the k-th keep the first in run order either way).  −1 when more than 64 entries are ≤ T_hi
// (the caller bisects the whole run).  r05: the whole-run bisection (32 steps × up to 16 ballots per wave, four
// resident blocks per CU sharing each SIMD's issue) was 13.4 of the kernel's ≈ 34 µs (tools/rr_stamps.py).
template <int J>
__device__ __forceinline__ int rws_select_narrow(const float *mk, const int *mp, int m, int k, float *tk, int *tp,
                                                 float *ok, int *op) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int nj = (m + 63) >> 6;
    unsigned u[J];
    unsigned mn = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int e = j * 64 + lane;
        u[j] = j < nj && e < m ? rws_bits(mk[e]) : 0xffffffffu;
        mn = min(mn, u[j]);
    }
    unsigned th = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const unsigned cand = th | (1u << bit);
        if ((int)__popcll(__ballot(mn < cand)) < k) th = cand;
    }
    int c = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const bool a = u[j] <= th && u[j] != 0xffffffffu;
        const unsigned long long ma = __ballot(a);
        const int p = c + (int)__popcll(ma & lt);
        if (a && p < 64) { tk[p] = mk[j * 64 + lane]; tp[p] = mp[j * 64 + lane]; }
        c += (int)__popcll(ma);
    }
    if (c > 64) return -1;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    unsigned dummy = 0;
    const unsigned T = rws_kth_bits<1>(tk, c, k, dummy);
    return rws_take<1>(tk, tp, c, k, T, ok, op);
}

template <int WV, int J>
__device__ __forceinline__ void rerank_wave_select(const float *__restrict__ pd, const int *__restrict__ pi,
                                                   int64_t total, int k, int64_t nrows, float bound,
                                                   float *wk, int *wp, float *sk, int *sp, int *scnt,
                                                   WaveList<1, int> &L, bool &bad, long long &rr_t, int64_t rr_q,
                                                   float *ntk, int *ntp) {
    (void)rr_t;
    (void)rr_q;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    float v[J];
    int r[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int64_t c = ((int64_t)j * WV + wv) * 64 + lane;
        v[j] = c < total ? pd[c] : __builtin_inff();
        r[j] = c < total ? pi[c] : -1;
    }
    RR_MARK(1);  // candidate loads issued
    float *mk = wk + wv * 64 * J;
    int *mp = wp + wv * 64 * J;
    int m = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        // NaN and +inf never; rows out of range never (pads)
        const bool a = v[j] <= bound && !(v[j] == __builtin_inff()) && r[j] >= 0 && r[j] < nrows;
        const unsigned long long ma = __ballot(a);
        if (a) { const int p = m + __popcll(ma & lt); mk[p] = v[j]; mp[p] = r[j]; }
        m += __popcll(ma);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the run's LDS writes before this wave reads it
    if constexpr (HIPANN_RR_STAMP != 0) { if (m >= 0) RR_STAMP_Q(rr_q, 6); }
    int kw;
    if (m <= k) {
        kw = m;
        for (int e = lane; e < m; e += 64) { sk[wv * 64 + e] = mk[e]; sp[wv * 64 + e] = mp[e]; }
    } else if (m <= 64) {  // one register of the run
        unsigned dummy = 0;
        const unsigned T = rws_kth_bits<1>(mk, m, k, dummy);
        kw = rws_take<1>(mk, mp, m, k, T, sk + wv * 64, sp + wv * 64);
    } else {
        kw = ntk ? rws_select_narrow<J>(mk, mp, m, k, ntk + wv * 64, ntp + wv * 64, sk + wv * 64, sp + wv * 64) : -1;
        if (kw < 0) {
            unsigned dummy = 0;
            const unsigned T = rws_kth_bits<J>(mk, m, k, dummy);
            kw = rws_take<J>(mk, mp, m, k, T, sk + wv * 64, sp + wv * 64);
        }
    }
    if (lane == 0) scnt[wv] = kw;
    RR_MARK(5);  // wave-local select
    RR_STAMP_Q(rr_q, 7);
    __syncthreads();
    if (wv != 0) return;
    // wave 0: the ≤ WV·k survivors, in wave order, compacted into its own run, then the k best
    int m0 = 0;
#pragma unroll
    for (int w = 0; w < WV; ++w) {
        const int n = scnt[w];
        const bool a = lane < n;
        float kk = a ? sk[w * 64 + lane] : 0.f;
        int pp = a ? sp[w * 64 + lane] : 0;
        if (a) { mk[m0 + lane] = kk; mp[m0 + lane] = pp; }
        m0 += n;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int nsel = m0;
    if (m0 > k && m0 <= 64) {  // (k <= 16: always) one register
        unsigned dummy = 0;
        const unsigned T = rws_kth_bits<1>(mk, m0, k, dummy);
        nsel = rws_take<1>(mk, mp, m0, k, T, sk, sp);  // wave 0's survivor slots are free again
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    } else if (m0 > k) {
        unsigned dummy = 0;
        const unsigned T = rws_kth_bits<WV>(mk, m0, k, dummy);
        nsel = rws_take<WV>(mk, mp, m0, k, T, sk, sp);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    } else {
        for (int e = lane; e < m0; e += 64) { sk[e] = mk[e]; sp[e] = mp[e]; }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    float kk = lane < nsel ? sk[lane] : __builtin_inff();
    int row = lane < nsel ? sp[lane] : IdTraits<int>::pad();
    wave_rank_sort(kk, row, nsel);
    bad = false;
    L.d[0] = lane < k ? kk : __builtin_inff();
    L.id[0] = lane < k ? row : IdTraits<int>::pad();
    RR_MARK(2);  // merge + sort
}

// ---------------------------------------------------------------------------------------------
// FAISS IndexIVFFlat's exact-tie membership.  Its scanner admits a candidate only when it is strictly
// better than the heap top (IVFFlatScanner: C::cmp(simi[0], dis)) and evicts the heap's worst by (key,
// label) (heap_replace_top's cmp2), scanning the probed lists in probe order and each list in row order.
// With T the k-th smallest key, that leaves exactly:
//   * every candidate with key < T (n_lt of them, n_lt < k), and
//   * of the candidates with key == T, those among the FIRST k candidates with key <= T in scan order
//     (the point where the heap top first reaches T; later T-keys are never admitted), of which the
//     k - n_lt smallest labels (each later admission evicted the largest-label T entry).
// Flat scans in label order, so there the rule is the plain (key, label) order; IVF lists are not
// label-ordered (duplicates stored under scattered ids, edge_cases.test:75-83).  ivf_scan_order_topk
// applies the rule to a candidate stream gen(c) -> (key, pos, label), c < n, pos = (probe rank << 32) |
// CSR row (scan order), keys +inf = no candidate, which must hold every candidate with key <= T (or
// the k - n_lt earliest T-keys per list: each list's candidates in row order): four passes of wave
// lists, the result in R as (key, label) ascending.
// ---------------------------------------------------------------------------------------------
struct ScanCand {
    float key;
    long long pos, label;
};

template <typename Gen>
__device__ __forceinline__ void ivf_scan_order_topk(int64_t n, int kout, Gen gen, WaveList<1, long long> &R) {
    const int lane = threadIdx.x & 63;
    const long long PAD = IdTraits<long long>::pad();
    // 1. the kout best by (key, scan position): T and n_lt
    WaveList<1, long long> A;
    A.init();
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        const ScanCand x = c0 + lane < n ? gen(c0 + lane) : ScanCand{__builtin_inff(), PAD, PAD};
        const bool ok = !(x.key == __builtin_inff());
        A.offer(ok ? x.key : __builtin_inff(), ok ? x.pos : PAD, kout - 1);
    }
    const float T = readlane_f(A.d[0], kout - 1);
    const bool full = !(T == __builtin_inff());
    const int n_lt = __popcll(__ballot(lane < kout && A.d[0] < T));
    // 2. the kout-th earliest scan position among keys <= T: the end of FAISS's admission window for T
    long long PM = PAD;
    if (full) {
        WaveList<1, long long> B;
        B.init();
        for (int64_t c0 = 0; c0 < n; c0 += 64) {
            const ScanCand x = c0 + lane < n ? gen(c0 + lane) : ScanCand{__builtin_inff(), PAD, PAD};
            const bool ok = x.key <= T;
            B.offer(ok ? 0.f : __builtin_inff(), ok ? x.pos : PAD, kout - 1);
        }
        PM = readlane_i(B.id[0], kout - 1);
    }
    // 3. the T-keys inside that window: their kout - n_lt smallest labels
    WaveList<1, long long> C;
    C.init();
    const int nt = kout - n_lt;
    if (full) {
        for (int64_t c0 = 0; c0 < n; c0 += 64) {
            const ScanCand x = c0 + lane < n ? gen(c0 + lane) : ScanCand{__builtin_inff(), PAD, PAD};
            const bool ok = x.key == T && x.pos <= PM;
            C.offer(ok ? 0.f : __builtin_inff(), ok ? x.label : PAD, nt - 1);
        }
    }
    // 4. the result: every key < T (all keys when fewer than kout), then the chosen T-keys; (key, label) order
    R.init();
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        const ScanCand x = c0 + lane < n ? gen(c0 + lane) : ScanCand{__builtin_inff(), PAD, PAD};
        const bool ok = !(x.key == __builtin_inff()) && (!full || x.key < T);
        R.offer(ok ? x.key : __builtin_inff(), ok ? x.label : PAD, kout - 1);
    }
    if (full) R.offer(lane < nt && C.id[0] != PAD ? T : __builtin_inff(), lane < nt ? C.id[0] : PAD, kout - 1);
}

// Probe rank of CSR row `row` for query q: its list (binary search of list_off) and that list's index among
// the query's nprobe probes (-1 if none).
__device__ __forceinline__ int ivf_probe_rank_of_row(int64_t row, const int64_t *__restrict__ list_off, int nlist,
                                                     const int64_t *__restrict__ qprobes, int nprobe) {
    int lo = 0, hi = nlist;  // list_off[lo] <= row < list_off[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (list_off[mid] <= row) lo = mid;
        else hi = mid;
    }
    for (int p = 0; p < nprobe; ++p)
        if (qprobes[p] == lo) return p;
    return -1;
}


// Re-run of one flagged query by one block (all WV waves): each probed list in probe order,
// every row's distance in the direct form (the same lane-strided fmaf chain and xor butterfly as
// rerank_rows4: the rerank's values bit for bit), a (distance, CSR row) list of kout per
// list into fpd/fpi[q][p][kout], then wave 0 applies FAISS's scan-order rule (ivf_scan_order_topk) and
// writes D/I.  The IVF rerank runs it with WV = 1 in the wave that flagged the query (no launch of its own).
template <bool IP, int WV>
__device__ __forceinline__ void ivf_block_fallback(int64_t q, int nprobe, int kout, const float *__restrict__ Q,
                                                const float *__restrict__ codes, int d, const int64_t *__restrict__ ids,
                                                int64_t label_offset, const int64_t *__restrict__ probes,
                                                const int64_t *__restrict__ list_off, const int *__restrict__ list_len,
                                                int nlist, float *__restrict__ fpd, long long *__restrict__ fpi,
                                                float *__restrict__ D, int64_t *__restrict__ I,
                                                unsigned long long *__restrict__ total, float *sd2, long long *si2) {
    // WV = 1: one wave on its own (the rerank's inline re-run): sd2 / si2 are that wave's 64 entries
    const int lane = threadIdx.x & 63, wv = WV == 1 ? 0 : threadIdx.x >> 6;
    const float *qp = Q + q * (int64_t)d;
    for (int p = 0; p < nprobe; ++p) {
        const int64_t l = probes[q * nprobe + p];
        WaveList<1, long long> L;
        L.init();
        if (l >= 0 && l < nlist && list_len[l] > 0) {
            const int64_t r0 = list_off[l], len = list_len[l];
            for (int64_t g = (int64_t)wv * 64; g < len; g += 64 * WV) {
                const int nr = (int)(len - g < 64 ? len - g : 64);
                float mine = __builtin_inff();
                for (int r = 0; r < nr; r += 4) {
                    float acc[4] = {0.f, 0.f, 0.f, 0.f};
                    const float *xr[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) xr[u] = codes + (r0 + g + (r + u < nr ? r + u : nr - 1)) * d;
                    for (int e = lane; e < d; e += 64) {
                        const float qv = qp[e];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const float xv = xr[u][e];
                            if (IP) acc[u] = fmaf(qv, xv, acc[u]);
                            else {
                                const float t = qv - xv;
                                acc[u] = fmaf(t, t, acc[u]);
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        float a = acc[u];
#pragma unroll
                        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
                        if (lane == r + u) mine = IP ? -a : a;
                    }
                }
                const bool ok = lane < nr && !(mine == __builtin_inff());
                L.offer(ok ? mine : __builtin_inff(), ok ? (long long)(r0 + g + lane) : IdTraits<long long>::pad(),
                        kout - 1);
            }
        }
        if constexpr (WV > 1) {
            sd2[wv * 64 + lane] = L.d[0];
            si2[wv * 64 + lane] = L.id[0];
            __syncthreads();
            if (wv == 0) {
                L.init();
#pragma unroll
                for (int w = 0; w < WV; ++w) L.offer(sd2[w * 64 + lane], si2[w * 64 + lane], kout - 1);
            }
        }
        if (wv == 0 && lane < kout) {
            fpd[(q * nprobe + p) * kout + lane] = L.d[0];
            fpi[(q * nprobe + p) * kout + lane] = L.id[0];
        }
        if constexpr (WV > 1) __syncthreads();
        else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // this wave's fpd stores land before its reads below
    }
    if (wv != 0) return;
    WaveList<1, long long> R;
    const int64_t n = (int64_t)nprobe * kout;
    const float *pd = fpd + q * n;
    const long long *pr = fpi + q * n;
    ivf_scan_order_topk(n, kout, [&](int64_t c) {
        const float key = pd[c];
        const long long row = pr[c];
        const bool ok = !(key == __builtin_inff()) && row != IdTraits<long long>::pad();
        const long long pp = c / kout;
        return ScanCand{ok ? key : __builtin_inff(), ok ? (pp << 32) | row : IdTraits<long long>::pad(),
                        ok ? (long long)(ids ? ids[row] : label_offset + row) : IdTraits<long long>::pad()};
    }, R);
    const float pad_d = IP ? -__builtin_inff() : __builtin_inff();
    if (lane < kout) {
        const bool pad = R.id[0] == IdTraits<long long>::pad() || R.d[0] == __builtin_inff();
        D[q * kout + lane] = pad ? pad_d : (IP ? -R.d[0] : R.d[0]);
        I[q * kout + lane] = pad ? -1 : (int64_t)R.id[0];
    }
    if (lane == 0) atomicAdd(total, 1ull);
}

// ---------------------------------------------------------------------------------------------
// ivf_fallback_chunks — the exact forms' flagged queries re-run in parallel (one launch after ivf_rerank_topk, every
// batch; it returns at once when nothing was flagged).  The rerank flags a query when its k-th reranked distance is not
// clear of the filter's bound; the first fb_cap of a batch's flagged queries come here: item (flagged query f, probe
// p, chunk c of chunk_rows rows of that probe's list) is one wave's work — the rows' direct-form distances in
// rerank_rows4's arithmetic (the rerank's values bit for bit), the chunk's kout best (distance, CSR row) into
// cpd/cpi[f][p][c].  Each wave counts its item on done[f] (its stores released at agent scope first: another XCD's
// wave may merge them); the wave whose add completes the query's count merges its candidates with FAISS's scan-order
// rule (ivf_scan_order_topk: probe rank, then CSR row) and writes D/I — the result ivf_block_fallback computes with
// one wave, at the parallelism of the chip (a flagged query over 200K-row lists took one wave 40 ms).
// ---------------------------------------------------------------------------------------------
template <bool IP>
__global__ void __launch_bounds__(256)
ivf_fallback_chunks(const int *__restrict__ nflag, const int *__restrict__ flagged, int fb_cap, int nprobe, int maxch,
                    int chunk_rows, int kout, const float *__restrict__ Q, const float *__restrict__ codes, int d,
                    const int64_t *__restrict__ ids, int64_t label_offset, const int64_t *__restrict__ probes,
                    const int64_t *__restrict__ list_off, const int *__restrict__ list_len, int nlist,
                    float *__restrict__ cpd, long long *__restrict__ cpi, unsigned *__restrict__ done,
                    float *__restrict__ D, int64_t *__restrict__ I, unsigned long long *__restrict__ total) {
    const int nf0 = *nflag;
    const int nf = nf0 < fb_cap ? nf0 : fb_cap;
    if (nf <= 0) return;
    const int lane = threadIdx.x & 63;
    const long long PAD = IdTraits<long long>::pad();
    const int64_t per_q = (int64_t)nprobe * maxch;  // item slots per flagged query
    const int64_t items = (int64_t)nf * per_q;
    const int64_t nw = (int64_t)gridDim.x * 4;
    // the list of probe p of query q, and its length (0: nothing to scan)
    auto plist = [&](int64_t q, int p, int64_t &l, int64_t &len) {
        l = probes[q * nprobe + p];
        len = l >= 0 && l < nlist ? (int64_t)list_len[l] : 0;
    };
    for (int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); it < items; it += nw) {
        const int f = (int)(it / per_q);
        const int p = (int)((it / maxch) % nprobe);
        const int c = (int)(it % maxch);
        const int64_t q = flagged[f];
        int64_t l, len;
        plist(q, p, l, len);
        const int64_t g0 = (int64_t)c * chunk_rows;
        if (g0 >= len) continue;  // an empty item: no candidates, not counted
        const int64_t g1 = len < g0 + chunk_rows ? len : g0 + chunk_rows, r0 = list_off[l];
        const float *qp = Q + q * (int64_t)d;
        WaveList<1, long long> L;
        L.init();
        for (int64_t g = g0; g < g1; g += 64) {
            const int nr = (int)(g1 - g < 64 ? g1 - g : 64);
            float mine = __builtin_inff();
            for (int r = 0; r < nr; r += 4) {
                float acc[4] = {0.f, 0.f, 0.f, 0.f};
                const float *xr[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) xr[u] = codes + (r0 + g + (r + u < nr ? r + u : nr - 1)) * d;
                rerank_rows4<IP>(qp, xr, d, lane, acc);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    float a = acc[u];
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
                    if (lane == r + u) mine = IP ? -a : a;
                }
            }
            const bool ok = lane < nr && !(mine == __builtin_inff());
            L.offer(ok ? mine : __builtin_inff(), ok ? (long long)(r0 + g + lane) : PAD, kout - 1);
        }
        if (lane < kout) {
            cpd[it * kout + lane] = L.d[0];
            cpi[it * kout + lane] = L.id[0];
        }
        // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): this wave's stores complete, are written back at
        // agent scope, then counted; the wave that completes the count acquires before reading any of them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(done + f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = (unsigned)__shfl((int)old, 0);
        // the query's non-empty items: Σ_p ⌈len_p / chunk_rows⌉
        int64_t need = 0;
        for (int pp = lane; pp < nprobe; pp += 64) {
            int64_t ll, ln;
            plist(q, pp, ll, ln);
            need += (ln + chunk_rows - 1) / chunk_rows;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) need += __shfl_xor(need, o);
        if ((int64_t)old + 1 != need) continue;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const float *pd = cpd + (int64_t)f * per_q * kout;
        const long long *pr = cpi + (int64_t)f * per_q * kout;
        int64_t lenv = 0;  // lane p < 64: probe p's list length (read by shuffle in the candidate stream)
        if (lane < nprobe) {
            int64_t ll;
            plist(q, lane, ll, lenv);
        }
        WaveList<1, long long> R;
        ivf_scan_order_topk(per_q * kout, kout, [&](int64_t cc) {
            const int64_t slot = cc / kout;  // p·maxch + chunk
            const int pp = (int)(slot / maxch);
            int64_t ll, ln;
            if (nprobe <= 64) ln = __shfl(lenv, pp);
            else plist(q, pp, ll, ln);
            const bool live = (slot % maxch) * (int64_t)chunk_rows < ln;  // empty items wrote nothing
            const float key = live ? pd[cc] : __builtin_inff();
            const long long row = live ? pr[cc] : PAD;
            const bool ok = !(key == __builtin_inff()) && row != PAD;
            return ScanCand{ok ? key : __builtin_inff(), ok ? ((long long)pp << 32) | row : PAD,
                            ok ? (long long)(ids ? ids[row] : label_offset + row) : PAD};
        }, R);
        const float pad_d = IP ? -__builtin_inff() : __builtin_inff();
        if (lane < kout) {
            const bool pad = R.id[0] == PAD || R.d[0] == __builtin_inff();
            D[q * kout + lane] = pad ? pad_d : (IP ? -R.d[0] : R.d[0]);
            I[q * kout + lane] = pad ? -1 : (int64_t)R.id[0];
        }
        if (lane == 0) {
            __hip_atomic_store(done + f, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next batch
            atomicAdd(total, 1ull);
        }
    }
}

void launch_ivf_fallback_chunks(const int *nflag, const int *flagged, int fb_cap, int nprobe, int maxch, int chunk_rows,
                                int kout, int metric, const float *Q, const float *codes, int d, const int64_t *ids,
                                int64_t label_offset, const int64_t *probes, const int64_t *list_off,
                                const int *list_len, int nlist, float *cpd, long long *cpi, unsigned *done, float *D,
                                int64_t *I, unsigned long long *total, hipStream_t st) {
    if (fb_cap <= 0) return;
    HIPANN_REQUIRE(kout >= 1 && kout <= 64 && maxch >= 1 && chunk_rows >= 64, "ivf fallback: arguments out of range");
    dim3 grid(256), block(256);  // 1024 waves: a grid-stride loop over the items; an empty batch returns at once
    if (metric == kIP)
        hipLaunchKernelGGL(ivf_fallback_chunks<true>, grid, block, 0, st, nflag, flagged, fb_cap, nprobe, maxch,
                           chunk_rows, kout, Q, codes, d, ids, label_offset, probes, list_off, list_len, nlist, cpd, cpi,
                           done, D, I, total);
    else
        hipLaunchKernelGGL(ivf_fallback_chunks<false>, grid, block, 0, st, nflag, flagged, fb_cap, nprobe, maxch,
                           chunk_rows, kout, Q, codes, d, ids, label_offset, probes, list_off, list_len, nlist, cpd, cpi,
                           done, D, I, total);
    HIPANN_CHECK(hipGetLastError());
}

#ifndef HIPANN_RR_MINB
#define HIPANN_RR_MINB 4  // 4-wave blocks resident per CU: ≤ 128 VGPRs, one round for a 1024-query batch
#endif
// ---------------------------------------------------------------------------------------------
// ivf_rerank_topk — form kFormSplit2Exact.  The 2-term split-bf16 scan (≈2⁻¹⁶ relative per product)
// only prunes; the results are exact.  Per query (one wave): merge the partial lists to the
// kRerankK = 16 best (scan key, row); recompute those rows' distances in the FAISS CPU scanner's
// direct form (Σ(q−x)², or −q·x for IP; fp32, IVFFlatScanner / fvec_L2sqr); order them by (distance,
// label) and write the first kout.
// Exactness check: every row the scan pruned has a scan key ≥ K16, the 16th merged key (slot lists,
// the running per-query bound and the merge all keep the 16 best), and |scan key − exact distance| ≤
// E = 2⁻¹²·(‖q‖² + max‖x‖²) (the dropped split terms, ≤ 3·2⁻¹⁶·‖q‖‖x‖ per q·x, doubled, plus fp32
// rounding of the norms and of both sums, with margin).  A query whose kout-th exact distance is not
// < K16 − E (or < −K16... for IP the same bound on −q·x) is flagged; IVF: the flagging wave re-runs the query at
// once in the direct form (ivf_block_fallback, fpd != nullptr); the Flat forms: the host's candidate rerank /
// 3-term path.  With fewer than 16 merged candidates nothing was pruned.
// The list length k (16; 32 for Flat IP, common.hpp) is the number of candidates reranked.
// rxmax >= 0 (Flat form kFlatBf16Exact: one plain bf16 product per element): the bound is the
// Cauchy-Schwarz bound of the bf16 rounding instead, from this query's own rounding residual and the
// largest row residual: |q̂·x̂ − q·x| ≤ ‖q‖·‖x̂−x‖ + ‖q̂−q‖·‖x̂‖ ≤ ‖q‖·rxmax + ‖q̂−q‖·(max‖x‖ + rxmax),
// plus the fp32 accumulation of d exact products (≤ d·2⁻²⁴·‖q̂‖‖x̂‖), doubled for L2, plus the fp32
// rounding of the key and of the reranked direct distance (≤ (d + 8)·2⁻²⁴·2(‖q‖² + max‖x‖²)), all ×1.01.
// ---------------------------------------------------------------------------------------------
// WV = 1: one wave per query, four queries per block (large batches).  WV > 1 (small batches, the
// extension's nq = 1 call): one block of WV waves per query — the waves merge disjoint parts of the
// partial lists and compute a share of the candidates' distances, wave 0 finishes.
template <bool IP, int WV>
__global__ void __launch_bounds__(WV == 1 ? 256 : 64 * WV, WV == 4 ? HIPANN_RR_MINB : 1)
ivf_rerank_topk(const float *__restrict__ pd, const int *__restrict__ pi, const int *__restrict__ slot_off,
                int nprobe, int64_t nq, int k, int kout, const float *__restrict__ Q,
                const float *__restrict__ codes, int d, const int64_t *__restrict__ ids, int64_t nrows,
                int64_t label_offset, float xmax2, float *__restrict__ D, int64_t *__restrict__ I,
                int *__restrict__ nflag, int *__restrict__ flagged, float eps, float rxmax,
                const float *__restrict__ qres, const int64_t *__restrict__ probes,
                const int64_t *__restrict__ list_off, int nlist, const unsigned *__restrict__ qbound,
                const float *__restrict__ qnorm, int kslot, int sub, const int *__restrict__ list_len,
                float *__restrict__ fpd, long long *__restrict__ fpi, unsigned long long *__restrict__ fb_total,
                int fb_cap) {
    const int64_t q = WV == 1 ? (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6) : (int64_t)blockIdx.x;
    if (q >= nq) return;
    const int lane = threadIdx.x & 63;
    const int wv = WV == 1 ? 0 : (int)(threadIdx.x >> 6);
    RR_STAMP(0);
    long long rr_t = HIPANN_RR_PROF ? clock64() : 0;
    // 1. the k best (scan key, row) of the query's partial lists (kslot entries per slot)
    WaveList<1, int> L;
    L.init();
    // slot_off == nullptr: the query's lists are the nprobe consecutive slots [q·nprobe, (q+1)·nprobe)
    // (the Flat exact form: one list per database split, query-major)
    const int64_t s0 = slot_off ? slot_off[q * nprobe] : q * nprobe;
    const int64_t s1 = slot_off ? slot_off[(q + 1) * nprobe] : (q + 1) * nprobe;
    const int64_t total = (s1 - s0) * kslot;
    if constexpr (HIPANN_RR_STAMP != 0) { if (total >= 0) RR_STAMP(1); }
    pd += s0 * kslot;
    pi += s0 * kslot;
    // sub-list slots (the IVF scans at request_k > 12, mf_finish_item): T_sub = qbound[q], the smallest k-th key
    // over the query's full sub-lists — every row a sub-list or the running bound pruned has scan key ≥ T_sub.
    // Candidates with key ≥ T_sub never matter when the check below passes (their exact distance is ≥ T_sub − E
    // > the kout-th), so they are not offered.
    float tsub = __builtin_inff();
    if (sub && qbound) {
        const unsigned b = qbound[q];
        const float t = __uint_as_float((b & 0x80000000u) ? (b & 0x7fffffffu) : ~b);
        tsub = t == t ? t : __builtin_inff();
    }
    // WV > 1 and ≤ 64·WV·RS_J candidates (block-uniform): the block's bitwise select (rerank_block_select)
    // instead of per-wave lists and serial inserts
    constexpr int RS_J = 16;
    const bool bsel = WV > 1 && total <= (int64_t)64 * WV * RS_J && !rerank_lists();
    if (WV > 1 && !bsel) RR_COUNT(9);
    constexpr int MU = 4;  // candidate chunks loaded ahead of their offers
    for (int64_t cb = (int64_t)wv * 64; !bsel && cb < total; cb += 64 * WV * MU) {
        float vv[MU];
        int rr[MU];
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const int64_t c = cb + (int64_t)u * 64 * WV + lane;
            vv[u] = c < total ? pd[c] : __builtin_inff();
            rr[u] = c < total ? pi[c] : -1;
        }
#pragma unroll
        for (int u = 0; u < MU; ++u) {
            const bool ok = rr[u] >= 0 && rr[u] < nrows && !(vv[u] == __builtin_inff()) && vv[u] < tsub;
            L.offer(ok ? vv[u] : __builtin_inff(), ok ? rr[u] : IdTraits<int>::pad(), k - 1);
        }
    }
    const float *qp = Q + q * (int64_t)d;
    float mine = __builtin_inff();
    int myrow, ncand;
    float k16;
    bool sel_bad = false;  // a selected candidate with an out-of-range row id (rerank_wave_select): flag the query
    // the per-query scalars of the bound check, loaded now (their latency hides under the candidate loads)
    const float qn_pre = qres && qnorm ? qnorm[q] : 0.f;
    const float qres_pre = qres ? qres[q] : 0.f;
    if constexpr (WV > 1) {
        __shared__ float sd[WV * 64], sdist[64];
        __shared__ int si[WV * 64], srow[64];
        __shared__ int scnt[2][WV];
        if (bsel) {
            // the scan's final bound (order-preserving bits of a full slot list's k-th key, atomicMin'ed): >= the
            // k-th smallest key of the query's candidates
            // (sub-lists: T_sub — the candidates above it are irrelevant, see above)
            float bound = __builtin_inff();
            if (sub) {
                bound = tsub;
            } else if (qbound) {
                const unsigned qb = qbound[q];
                const float t = __uint_as_float((qb & 0x80000000u) ? (qb & 0x7fffffffu) : ~qb);
                bound = t == t ? t : __builtin_inff();
            }
            RR_MARK(0);
#if HIPANN_RR_OLDSEL
            rerank_block_select<WV, RS_J>(pd, pi, total, k, nrows, sd, si, scnt, L, bound, rr_t);
#else
            __shared__ float wk[WV * 64 * RS_J];
            __shared__ int wp[WV * 64 * RS_J];
            __shared__ float ntk[WV * 64];
            __shared__ int ntp[WV * 64];
            rerank_wave_select<WV, RS_J>(pd, pi, total, k, nrows, bound, wk, wp, sd, si, scnt[0], L, sel_bad, rr_t, q,
                                         ntk, ntp);
#endif
            if (wv == 0) srow[lane] = lane < k ? L.id[0] : IdTraits<int>::pad();
            RR_STAMP(2);
        } else {
            sd[wv * 64 + lane] = lane < k ? L.d[0] : __builtin_inff();
            si[wv * 64 + lane] = lane < k ? L.id[0] : IdTraits<int>::pad();
            __syncthreads();
            if (wv == 0) {
                L.init();
#pragma unroll
                for (int w = 0; w < WV; ++w) L.offer(sd[w * 64 + lane], si[w * 64 + lane], k - 1);
                srow[lane] = lane < k ? L.id[0] : IdTraits<int>::pad();
            }
        }
        __syncthreads();
        // every wave: its share of the candidates' direct-form distances (4 rows in flight)
        for (int r0 = wv * 4; r0 < k; r0 += 4 * WV) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            const float *xr[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = r0 + u < k ? r0 + u : k - 1;
                const int row = srow[r];
                ok[u] = r0 + u < k && row != IdTraits<int>::pad();
                xr[u] = codes + (int64_t)(ok[u] ? row : 0) * d;
            }
            rerank_rows4<IP>(qp, xr, d, lane, acc);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float a = acc[u];
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
                if (lane == 0 && ok[u]) sdist[r0 + u] = IP ? -a : a;
            }
        }
        __syncthreads();
        RR_STAMP(3);
        RR_MARK(3);  // distances
        if (wv != 0) return;
        myrow = L.id[0];
        ncand = __popcll(__ballot(lane < k && myrow != IdTraits<int>::pad()));
        k16 = readlane_f(L.d[0], k - 1);
        if (lane < ncand) mine = sdist[lane];
    } else {
        myrow = L.id[0];
        ncand = __popcll(__ballot(lane < k && myrow != IdTraits<int>::pad()));
        k16 = readlane_f(L.d[0], k - 1);  // K_k: the k-th merged scan key
    }
    const bool real = lane < k && myrow != IdTraits<int>::pad();
    // 2. exact direct-form distances of the candidates (4 rows in flight, wave reduction per row)
    float qq = 0.f, rq2 = 0.f;
    if (qres && qnorm) {
        qq = qn_pre;  // the IVF fp16 form: ‖q‖² prepared with the query terms, its own split residual in qres
    } else {
        int e = lane;
        for (; e + 192 < d; e += 256) {  // 4 strides of loads in flight, sums in e order
            float qv[4];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) qv[s2] = qp[e + 64 * s2];
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                qq = fmaf(qv[s2], qv[s2], qq);
                const float r = qv[s2] - (float)(__bf16)qv[s2];  // RNE, as the bf16 image of the queries
                rq2 = fmaf(r, r, rq2);
            }
        }
        for (; e < d; e += 64) {
            qq = fmaf(qp[e], qp[e], qq);
            const float r = qp[e] - (float)(__bf16)qp[e];
            rq2 = fmaf(r, r, rq2);
        }
    }
    if (!(qres && qnorm)) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            qq += __shfl_xor(qq, o);
            rq2 += __shfl_xor(rq2, o);
        }
    }
    if constexpr (WV == 1) {
    for (int r0 = 0; r0 < ncand; r0 += 4) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float *xr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = r0 + u < ncand ? r0 + u : ncand - 1;
            xr[u] = codes + (int64_t)__builtin_amdgcn_readlane(myrow, r) * d;
        }
        rerank_rows4<IP>(qp, xr, d, lane, acc);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float a = acc[u];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
            if (lane == r0 + u) mine = IP ? -a : a;
        }
    }
    }
    // 3. (distance, label) order, first kout
    WaveList<1, long long> R;
    const long long lab = real ? (long long)(ids ? ids[myrow] : label_offset + myrow) : IdTraits<long long>::pad();
    {
        // the ncand reranked candidates sit in lanes < ncand: their (distance, label) order by rank (no insert chain)
        float rk = real ? mine : __builtin_inff();
        long long rl = lab;
        wave_rank_sort(rk, rl, ncand);
        R.d[0] = rk;
        R.id[0] = rl;
    }
    // 3b. exact ties at the kout-th distance with more tied rows than slots left: FAISS's scan-order
    // admission decides which tied labels stay (ivf_scan_order_topk).  Every row with distance <= the
    // kout-th is among the candidates whenever the bound check below passes (they all have scan key
    // <= dk + E < K16); a flagged query is redone by the fallback, which applies the same rule.
    if (probes) {
        const float T = readlane_f(R.d[0], kout - 1);
        const int n_le = __popcll(__ballot(real && mine <= T));
        if (!(T == __builtin_inff()) && n_le > kout) {
            const int64_t pr = real && mine <= T
                                   ? ivf_probe_rank_of_row(myrow, list_off, nlist, probes + q * nprobe, nprobe) : -1;
            const long long pos = pr >= 0 ? ((long long)pr << 32) | (long long)myrow : IdTraits<long long>::pad();
            const float mk = real ? mine : __builtin_inff();
            ivf_scan_order_topk(64, kout, [&](int64_t) { return ScanCand{mk, pos, lab}; }, R);
        }
    }
    if constexpr (WV > 1) RR_MARK(4);  // (distance, label) order + tie rule
    RR_STAMP(4);
    // 4. exactness check
    const float dk = readlane_f(R.d[0], kout - 1);
    float E;
    if (rxmax >= 0.f) {
        // qres (IVF fp16 form): the query's own split residual, and 2d products per accumulator chain
        const float qn = sqrtf(qq), rq = qres ? qres_pre : sqrtf(rq2), xh = sqrtf(xmax2) + rxmax;
        const float g = (float)(qres ? 2 * d : d) * 0x1p-24f;
        const float eip = qn * rxmax + rq * xh + g * (qn + rq) * xh;
        E = 1.01f * ((IP ? 1.f : 2.f) * eip + (float)(d + 8) * 0x1p-24f * 2.f * (qq + xmax2));
    } else {
        E = eps * (qq + xmax2);
    }
    // a non-finite bound (a query outside the fp16 form's safe scale range) is always re-run — unless the query
    // has no candidate at all: empty probe lists, or the Flat bounded passes' overflowed query, which
    // flat_cand_select already flagged (flagged holds nq entries: no query may be appended twice); sub-lists: the
    // kout-th distance must also clear the smallest full sub-list's k-th key
    const bool flag = sel_bad || (ncand > 0 && !(E <= 3.4e38f)) || (ncand == k && !(dk < k16 - E)) ||
                      (sub && tsub < __builtin_inff() && !(dk < tsub - E));
    int fslot = 0;
    if (flag && lane == 0) {
        fslot = atomicAdd(nflag, 1);
        flagged[fslot] = (int)q;
    }
    fslot = __shfl(fslot, 0);
    const float pad_d = IP ? -__builtin_inff() : __builtin_inff();
    // IVF: the first fb_cap flagged queries of the batch are re-run by ivf_fallback_chunks (the next launch: every
    // (query, probe, 2048-row chunk) by its own wave — a flagged query over long lists is no longer one wave's
    // serial scan); this wave writes its uncertified answer, which that kernel overwrites.  Later ones re-run here.
    if (flag && fpd && fslot >= fb_cap) {
        // IVF: this wave re-runs the query at once over its probe lists in the direct form with FAISS's scan-order
        // tie rule (the device fallback, ivf_block_fallback) — no separate launch per batch
        __shared__ float fsd[4 * 64];
        __shared__ long long fsi[4 * 64];
        const int pw = (int)(threadIdx.x >> 6);
        ivf_block_fallback<IP, 1>(q, nprobe, kout, Q, codes, d, ids, label_offset, probes, list_off, list_len, nlist,
                                  fpd, fpi, D, I, fb_total, fsd + pw * 64, fsi + pw * 64);
        return;
    }
    if (lane < kout) {
        const bool pad = R.id[0] == IdTraits<long long>::pad();
        D[q * kout + lane] = pad ? pad_d : (IP ? -R.d[0] : R.d[0]);
        I[q * kout + lane] = pad ? -1 : (int64_t)R.id[0];
    }
    RR_STAMP(5);
    if constexpr (WV > 1) {
        RR_MARK(8);  // bound check + write
#if HIPANN_RR_PROF
        if (lane == 0) atomicAdd(&rr_prof[7], 1ull);
#endif
    }
}

// ---------------------------------------------------------------------------------------------
// Flat form 4, second stage for the flagged queries (flat_cand_rerank_part / _final).  The bounded passes
// buffered EVERY row whose scan key is ≤ the pass bound T = bound[q] (pass A under T₀ ≥ T, pass B under T),
// so a row outside the buffers has scan key > T and exact distance > T − E.  Recomputing all of a flagged
// query's buffered rows in the direct form (≈ 26 per split at 10M rows) and ordering them by (distance,
// label) gives its exact top-kout whenever the kout-th distance is < T − E: T is the 32nd best key of pass
// A's ≈ 1/20 of the rows, far looser than the 32nd best key overall that the first rerank had to clear
// (flat_cand_select).  A query with an overflowed cell, or that fails this check too, goes to flagged2
// (the SPLIT3 re-run).  part: grid (nf, P) blocks, wave w of block p takes splits p·spb + w, + 4, …; each
// wave keeps a (distance, label) list of kout, the block merges its 4 lists; final: one wave per query.
// ---------------------------------------------------------------------------------------------
constexpr int kCandRerankParts = 16;
template <bool IP>
__global__ void __launch_bounds__(256)
flat_cand_rerank_part(const int *__restrict__ flagged, const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                      const int *__restrict__ cand_n, int nsplit, int cap, const float *__restrict__ Q,
                      const float *__restrict__ X, int d, int64_t nrows, int64_t label_offset, int kout,
                      float *__restrict__ part_d, long long *__restrict__ part_i, int *__restrict__ ovf) {
    __shared__ float sd[4][64];
    __shared__ long long si[4][64];
    const int f = blockIdx.x, p = blockIdx.y, P = gridDim.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t q = flagged[f];
    const float *qp = Q + q * (int64_t)d;
    const int spb = (nsplit + P - 1) / P;
    const int s_begin = p * spb, s_end = nsplit < s_begin + spb ? nsplit : s_begin + spb;
    WaveList<1, long long> L;
    L.init();
    bool over = false;
    for (int s = s_begin + wv; s < s_end; s += 4) {
        const int64_t cell = q * nsplit + s;
        const int nr = cand_n[cell];
        over |= nr > cap;
        const int n = nr < cap ? nr : cap;
        for (int r0 = 0; r0 < n; r0 += 4) {
            const float *xr[4];
            int row[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = r0 + u < n ? r0 + u : n - 1;
                const int rw = cand_i[cell * cap + j];
                row[u] = r0 + u < n && rw >= 0 && rw < nrows ? rw : -1;
                xr[u] = X + (int64_t)(row[u] >= 0 ? row[u] : 0) * d;
            }
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            rerank_rows4<IP>(qp, xr, d, lane, acc);
            float mine = __builtin_inff();
            long long lab = IdTraits<long long>::pad();
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float a = acc[u];
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
                if (lane == u && row[u] >= 0) { mine = IP ? -a : a; lab = label_offset + row[u]; }
            }
            L.offer(mine, lab, kout - 1);
        }
    }
    sd[wv][lane] = L.d[0];
    si[wv][lane] = L.id[0];
    const bool bover = __syncthreads_or(over);
    if (wv != 0) return;
#pragma unroll
    for (int w = 1; w < 4; ++w) L.offer(lane < kout ? sd[w][lane] : __builtin_inff(),
                                        lane < kout ? si[w][lane] : IdTraits<long long>::pad(), kout - 1);
    if (lane < kout) {
        part_d[((int64_t)f * P + p) * kout + lane] = L.d[0];
        part_i[((int64_t)f * P + p) * kout + lane] = L.id[0];
    }
    if (lane == 0) ovf[f * P + p] = bover ? 1 : 0;
}

template <bool IP>
__global__ void __launch_bounds__(64)
flat_cand_rerank_final(const int *__restrict__ flagged, int P, const float *__restrict__ bound,
                       const float *__restrict__ Q, int d, float xmax2, float rxmax, int kout,
                       const float *__restrict__ part_d, const long long *__restrict__ part_i,
                       const int *__restrict__ ovf, float *__restrict__ D, int64_t *__restrict__ I,
                       int *__restrict__ nflag2, int *__restrict__ flagged2, float *__restrict__ dbg,
                       const float *__restrict__ qres) {
    const int f = blockIdx.x, lane = threadIdx.x;
    const int64_t q = flagged[f];
    bool over = false;
    for (int p = 0; p < P; ++p) over |= ovf[f * P + p] != 0;
    WaveList<1, long long> L;
    L.init();
    for (int p = 0; p < P; ++p)
        L.offer(lane < kout ? part_d[((int64_t)f * P + p) * kout + lane] : __builtin_inff(),
                lane < kout ? part_i[((int64_t)f * P + p) * kout + lane] : IdTraits<long long>::pad(), kout - 1);
    // the bound of the first rerank (ivf_rerank_topk, rxmax >= 0 branch) from this query's own norms
    const float *qp = Q + q * (int64_t)d;
    float qq = 0.f, rq2 = 0.f;
    for (int e = lane; e < d; e += 64) {
        qq = fmaf(qp[e], qp[e], qq);
        const float r = qp[e] - (float)(__bf16)qp[e];
        rq2 = fmaf(r, r, rq2);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        qq += __shfl_xor(qq, o);
        rq2 += __shfl_xor(rq2, o);
    }
    // qres (the int8 form): the query's own int8 residual, and 2d terms of accumulation margin as the first rerank
    const float qn = sqrtf(qq), rq = qres ? qres[q] : sqrtf(rq2), xh = sqrtf(xmax2) + rxmax;
    const float g = (float)(qres ? 2 * d : d) * 0x1p-24f;
    const float eip = qn * rxmax + rq * xh + g * (qn + rq) * xh;
    const float T = bound[q];
    // + 2^-20 of the key scale: the pass compared s against ‖q‖² − T (IP: −2T) in fp32
    const float E = 1.01f * ((IP ? 1.f : 2.f) * eip + (float)(d + 8) * 0x1p-24f * 2.f * (qq + xmax2)) +
                    0x1p-20f * (qq + xmax2 + fabsf(T));
    const float dk = readlane_f(L.d[0], kout - 1);
    const bool ok = !over && E <= 3.4e38f && dk < __builtin_inff() && (T == __builtin_inff() || dk < T - E);
    if (dbg && lane == 0) {  // HIPANN_FLAT_CAND_DEBUG: (overflow, k-th distance, pass bound, E) per flagged query
        dbg[4 * f + 0] = over ? 1.f : 0.f;
        dbg[4 * f + 1] = dk;
        dbg[4 * f + 2] = T;
        dbg[4 * f + 3] = E;
    }
    if (!ok) {
        if (lane == 0) flagged2[atomicAdd(nflag2, 1)] = (int)q;
        return;
    }
    if (lane < kout) {
        D[q * kout + lane] = IP ? -L.d[0] : L.d[0];
        I[q * kout + lane] = (int64_t)L.id[0];
    }
}

void launch_flat_cand_rerank(const int *flagged, int nf, const float *cand_d, const int *cand_i, const int *cand_n,
                             int nsplit, int cap, const float *bound, const float *Q, const float *X, int d,
                             int64_t nrows, int64_t label_offset, float xmax2, float rxmax, int metric, int kout,
                             float *part_d, long long *part_i, int *ovf, float *D, int64_t *I, int *nflag2,
                             int *flagged2, hipStream_t st, float *dbg, const float *qres) {
    if (nf <= 0) return;
    HIPANN_REQUIRE(kout >= 1 && kout <= 64 && nsplit >= 1 && cap >= 1, "flat cand rerank: bad arguments");
    const int P = std::min(kCandRerankParts, nsplit);
    dim3 g1((unsigned)nf, (unsigned)P);
    if (metric == kIP) {
        hipLaunchKernelGGL(flat_cand_rerank_part<true>, g1, dim3(256), 0, st, flagged, cand_d, cand_i, cand_n, nsplit,
                           cap, Q, X, d, nrows, label_offset, kout, part_d, part_i, ovf);
        hipLaunchKernelGGL(flat_cand_rerank_final<true>, dim3((unsigned)nf), dim3(64), 0, st, flagged, P, bound, Q, d,
                           xmax2, rxmax, kout, part_d, part_i, ovf, D, I, nflag2, flagged2, dbg, qres);
    } else {
        hipLaunchKernelGGL(flat_cand_rerank_part<false>, g1, dim3(256), 0, st, flagged, cand_d, cand_i, cand_n, nsplit,
                           cap, Q, X, d, nrows, label_offset, kout, part_d, part_i, ovf);
        hipLaunchKernelGGL(flat_cand_rerank_final<false>, dim3((unsigned)nf), dim3(64), 0, st, flagged, P, bound, Q, d,
                           xmax2, rxmax, kout, part_d, part_i, ovf, D, I, nflag2, flagged2, dbg, qres);
    }
    HIPANN_CHECK(hipGetLastError());
}

int flat_cand_rerank_parts(int nsplit) { return std::min(kCandRerankParts, nsplit); }

// max over rows of ‖x‖² (non-negative floats order as their bit patterns)
__global__ void __launch_bounds__(256) ivf_max_norm(const float *__restrict__ xn, int64_t n, unsigned *__restrict__ out) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) m = fmaxf(m, xn[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

__global__ void __launch_bounds__(256) ivf_gather_queries(const float *__restrict__ Q, const int *__restrict__ idx, int nf,
                                                          int d, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nf * d) return;
    const int j = (int)(t / d), e = (int)(t - (int64_t)j * d);
    out[t] = Q[(int64_t)idx[j] * d + e];
}

__global__ void __launch_bounds__(256) ivf_scatter_results(const float *__restrict__ Df, const int64_t *__restrict__ If,
                                                           const int *__restrict__ idx, int nf, int kout,
                                                           float *__restrict__ D, int64_t *__restrict__ I) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nf * kout) return;
    const int j = (int)(t / kout), e = (int)(t - (int64_t)j * kout);
    D[(int64_t)idx[j] * kout + e] = Df[t];
    I[(int64_t)idx[j] * kout + e] = If[t];
}

#ifndef HIPANN_RR_WIDE
#define HIPANN_RR_WIDE (1 << 30)  // below this many queries: one 4-wave block per query (nq 1024: 80 -> 65 us)
#endif

void launch_ivf_rerank(const float *pd, const int *pi, const int *slot_off, int nprobe, int64_t nq, int k, int kout,
                       int metric, const float *Q, const float *codes, int d, const int64_t *ids, int64_t nrows,
                       int64_t label_offset, float xmax2, float *D, int64_t *I, int *nflag, int *flagged,
                       hipStream_t st, float eps, float rxmax, const float *qres, const int64_t *probes,
                       const int64_t *list_off, int nlist, const unsigned *qbound, const float *qnorm, int kslot,
                       int sub, const int *list_len, float *fpd, long long *fpi, unsigned long long *fb_total,
                       int fb_cap) {
    if (nq <= 0) return;
    if (kslot <= 0) kslot = k;
    // the filter depth k bounds kout (kout = k leaves no margin: those queries are flagged and re-run exactly)
    HIPANN_REQUIRE(k >= kRerankK && k <= 64 && kout >= 1 && kout <= k && kslot >= 1 && (!sub || qbound),
                   "ivf rerank: k / kout out of range");
    HIPANN_REQUIRE(!fpd || (fpi && list_len && probes && list_off && fb_total), "ivf rerank: inline re-run buffers");
    // small batches: one 4-wave block per query (fills more of the chip, shorter per-query chain)
    const bool wide = nq < HIPANN_RR_WIDE;
    dim3 grid((unsigned)(wide ? nq : ceil_div(nq, 4))), block(256);
#define RR_ARGS pd, pi, slot_off, nprobe, nq, k, kout, Q, codes, d, ids, nrows, label_offset, xmax2, D, I, nflag, flagged, \
                eps, rxmax, qres, probes, list_off, nlist, qbound, qnorm, kslot, sub, list_len, fpd, fpi, fb_total, \
                fpd ? fb_cap : 0
    if (metric == kIP) {
        if (wide) hipLaunchKernelGGL((ivf_rerank_topk<true, 4>), grid, block, 0, st, RR_ARGS);
        else hipLaunchKernelGGL((ivf_rerank_topk<true, 1>), grid, block, 0, st, RR_ARGS);
    } else {
        if (wide) hipLaunchKernelGGL((ivf_rerank_topk<false, 4>), grid, block, 0, st, RR_ARGS);
        else hipLaunchKernelGGL((ivf_rerank_topk<false, 1>), grid, block, 0, st, RR_ARGS);
    }
#undef RR_ARGS
    HIPANN_CHECK(hipGetLastError());
}

// tuning builds (HIPANN_RR_PROF): the wide rerank's wave-0 clock sums per phase — [0] setup, [1] candidate loads,
// [5] bound count, [2] compaction / search + sort, [3] distances, [4] order + ties, [8] bound check + write — and the
// counts [6] compaction path, [9] list path, [7] queries (16 entries); reset after reading
// tuning builds (HIPANN_RR_STAMP): per query q < 4096 eight s_memrealtime stamps (100 MHz) — [0] entry, [1] slot range
// known, [6] candidates loaded and compacted, [7] wave 0's wave-local select done, [2] candidates selected,
// [3] distances done, [4] order done, [5] written (tools/rr_stamps.py)
extern "C" int hipann_debug_rr_stamps(long long *out, int n) {
#if HIPANN_RR_STAMP
    if (n > 4096 * 8 || hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(rr_stamp), sizeof(long long) * (size_t)n) == hipSuccess ? 0 : -1;
#else
    (void)out;
    (void)n;
    return -1;
#endif
}

extern "C" int hipann_debug_rr_prof(unsigned long long *out16) {
#if HIPANN_RR_PROF
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(rr_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rr_prof), z, sizeof z) != hipSuccess) return -1;
    return 0;
#else
    (void)out16;
    return -1;
#endif
}

void launch_ivf_max_norm(const float *xn, int64_t n, unsigned *out, hipStream_t st) {
    HIPANN_CHECK(hipMemsetAsync(out, 0, sizeof(unsigned), st));
    if (n <= 0) return;
    const unsigned blocks = (unsigned)std::min<int64_t>(1024, ceil_div(n, 256));
    hipLaunchKernelGGL(ivf_max_norm, dim3(blocks), dim3(256), 0, st, xn, n, out);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_gather_queries(const float *Q, const int *idx, int nf, int d, float *out, hipStream_t st) {
    if (nf <= 0) return;
    hipLaunchKernelGGL(ivf_gather_queries, dim3((unsigned)ceil_div((int64_t)nf * d, 256)), dim3(256), 0, st, Q, idx, nf,
                       d, out);
    HIPANN_CHECK(hipGetLastError());
}

void launch_ivf_scatter_results(const float *Df, const int64_t *If, const int *idx, int nf, int kout, float *D,
                                int64_t *I, hipStream_t st) {
    if (nf <= 0) return;
    hipLaunchKernelGGL(ivf_scatter_results, dim3((unsigned)ceil_div((int64_t)nf * kout, 256)), dim3(256), 0, st, Df, If,
                       idx, nf, kout, D, I);
    HIPANN_CHECK(hipGetLastError());
}

}  // namespace hipann
