// ivf_train.hip — IVF training (k-means) on the GPU behind the C ABI (hipann_ivf_train*, include/hip_ann.h).
//
// The extension trains its IndexIVFFlat on the CPU at CREATE INDEX: a deterministic stride sample of
// train_sample rows (src/faiss_index.cpp:302-319), then faiss_idx->train → FAISS 1.13.2 IndexIVF::train_q1 →
// Clustering::train (external): at most 256 points per centroid, an init from the training points, niter = 25
// Lloyd iterations of (assign with the flat quantizer, mean of each cluster, split empty clusters, spherical
// renormalisation for IP).  This file runs that pipeline with the training rows resident in HBM:
//   * assignment: the Flat search itself (flat_shard_search, k = 1, exact fp32 products — the coarse
//     quantizer's form), 65536 rows per call;
//   * cluster sums: a stable radix sort of (assignment, row) (rocPRIM), then one block per centroid summing its
//     rows in ascending row order in fp64 (deterministic, the oracle's order);
//   * k-means++ init (optional, the default): three launches per centre with no host round trip — fp64 D²
//     (wave per row: 64 lane-strided partials + xor butterfly), integer weights floor(D²·2^32/max D²) and their
//     per-block sums, one block drawing the row (t = r mod Σw: the same row whatever order the weights are
//     summed in) and copying it into the centre table;
//   * the per-iteration finish (means from the fp64 sums, FAISS's split_clusters, spherical renorm) on the host:
//     nlist × d values, the random draws from the same splitmix64 stream as the oracle.
// oracle/oracle.c oracle_kmeans_train restates exactly this; tests/test_ivf_train_gpu.py checks the two agree.
#include "../../include/hip_ann.h"
#include "ivf.hpp"

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

namespace hipann {

namespace {

uint64_t km_next(uint64_t &s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
float km_rand_float(uint64_t &s) { return (float)(km_next(s) >> 40) * 0x1p-24f; }

// ---- k-means++ -----------------------------------------------------------------------------------------
// d2[i] = min(d2[i], ‖T_i − c‖²) in fp64 (lane l sums dims l, l + 64, … in order; xor butterfly), and the max
// over rows as the bits of a non-negative double (atomicMax orders them like the values).
__global__ void __launch_bounds__(256) kpp_update(const float *__restrict__ T, int64_t m, int d,
                                                  const float *__restrict__ c, double *__restrict__ d2,
                                                  unsigned long long *__restrict__ maxbits) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    double v = 0.0;
    if (i < m) {
        const float *x = T + i * (int64_t)d;
        double acc = 0.0;
        for (int e = lane; e < d; e += 64) {
            const double df = (double)x[e] - (double)c[e];
            acc = acc + df * df;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc = acc + __shfl_xor(acc, o);
        const double old = d2[i];
        v = acc < old ? acc : old;
        if (lane == 0) d2[i] = v;
    }
    unsigned long long b = i < m ? (unsigned long long)__double_as_longlong(v) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = (unsigned long long)__shfl_xor((long long)b, o);
        b = t > b ? t : b;
    }
    if (lane == 0 && i < m) atomicMax(maxbits, b);
}

__device__ __forceinline__ unsigned long long kpp_weight(double d2, double scale) {
    return (unsigned long long)(d2 * scale);
}

// per-block sums of the integer weights w = floor(d2 · 2^32 / max); 256 rows per block
__global__ void __launch_bounds__(256) kpp_weights(const double *__restrict__ d2, int64_t m,
                                                   const unsigned long long *__restrict__ maxbits,
                                                   unsigned long long *__restrict__ bsum) {
    __shared__ unsigned long long part[4];
    const double mx = __longlong_as_double((long long)*maxbits);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long w = 0;
    if (i < m && mx > 0.0) w = kpp_weight(d2[i], 4294967296.0 / mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w += (unsigned long long)__shfl_xor((long long)w, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one block: t = r mod Σw, the first row whose running weight exceeds t (all weights zero: r mod m), its row
// copied into centre j; the max is reset for the next centre
__global__ void __launch_bounds__(256) kpp_pick(const double *__restrict__ d2, int64_t m,
                                                unsigned long long *__restrict__ maxbits,
                                                const unsigned long long *__restrict__ bsum, int nb,
                                                unsigned long long r, const float *__restrict__ T, int d,
                                                float *__restrict__ cen) {
    __shared__ long long pick;
    if (threadIdx.x == 0) {
        const double mx = __longlong_as_double((long long)*maxbits);
        long long p = (long long)(r % (unsigned long long)m);
        if (mx > 0.0) {
            unsigned long long tot = 0;
            for (int b = 0; b < nb; ++b) tot += bsum[b];
            if (tot > 0) {
                const unsigned long long t = r % tot;
                const double scale = 4294967296.0 / mx;
                unsigned long long acc = 0;
                int b = 0;
                for (; b < nb - 1 && acc + bsum[b] <= t; ++b) acc += bsum[b];
                p = m - 1;
                for (int64_t i = (int64_t)b * 256; i < m; ++i) {
                    acc += kpp_weight(d2[i], scale);
                    if (acc > t) { p = i; break; }
                }
            }
        }
        pick = p;
        *maxbits = 0ull;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < d; e += 256) cen[e] = T[pick * (int64_t)d + e];
}

__global__ void __launch_bounds__(256) km_fill_d2(double *__restrict__ d2, int64_t m) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < m) d2[i] = DBL_MAX;
}

// ---- Lloyd ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) km_keys(const int64_t *__restrict__ I, int64_t m, int nlist,
                                               unsigned *__restrict__ key, unsigned *__restrict__ val,
                                               int *__restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const int64_t a = I[i];
    const unsigned k = a >= 0 && a < nlist ? (unsigned)a : (unsigned)nlist;  // unassigned (cannot happen) last
    key[i] = k;
    val[i] = (unsigned)i;
    if (k < (unsigned)nlist) atomicAdd(cnt + k, 1);
}

// S[c][e] = Σ over the cluster's rows in ascending row order of T[row][e], in fp64
__global__ void __launch_bounds__(256) km_sums(const float *__restrict__ T, int d, const unsigned *__restrict__ rows,
                                               const int64_t *__restrict__ off, double *__restrict__ S) {
    const int c = blockIdx.x;
    const int64_t r0 = off[c], r1 = off[c + 1];
    for (int e = threadIdx.x; e < d; e += 256) {
        double acc = 0.0;
        for (int64_t j = r0; j < r1; ++j) acc = acc + (double)T[(int64_t)rows[j] * d + e];
        S[(int64_t)c * d + e] = acc;
    }
}

__global__ void __launch_bounds__(256) km_gather(const float *__restrict__ x, const int64_t *__restrict__ rows,
                                                 int64_t m, int d, float *__restrict__ T) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= m * d) return;
    const int64_t i = t / d, e = t - i * d;
    T[t] = x[rows[i] * (int64_t)d + e];
}

// Training rows: the reference's stride sample, then (above 256·nlist) a uniform subset in ascending order —
// oracle_kmeans_train steps 1-2, consuming the same draws.
std::vector<int64_t> training_rows(int64_t n, int64_t train_sample, int nlist, uint64_t &rs) {
    std::vector<int64_t> rows;
    if (train_sample > 0 && train_sample < n) {
        rows.resize((size_t)train_sample);
        const double stride = (double)n / (double)train_sample;
        for (int64_t i = 0; i < train_sample; ++i) rows[(size_t)i] = (int64_t)((double)i * stride);
    } else {
        rows.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) rows[(size_t)i] = i;
    }
    const int64_t m = (int64_t)rows.size();
    HIPANN_REQUIRE(m >= nlist, "ivf train: fewer training points than centroids");
    const int64_t maxp = (int64_t)256 * nlist;
    if (m > maxp) {
        std::vector<int64_t> perm((size_t)m);
        for (int64_t i = 0; i < m; ++i) perm[(size_t)i] = i;
        for (int64_t i = 0; i < maxp; ++i) {
            const int64_t j = i + (int64_t)(km_next(rs) % (uint64_t)(m - i));
            std::swap(perm[(size_t)i], perm[(size_t)j]);
        }
        std::vector<char> pick((size_t)m, 0);
        for (int64_t i = 0; i < maxp; ++i) pick[(size_t)perm[(size_t)i]] = 1;
        int64_t w = 0;
        for (int64_t i = 0; i < m; ++i)
            if (pick[(size_t)i]) rows[(size_t)w++] = rows[(size_t)i];
        rows.resize((size_t)maxp);
    }
    return rows;
}

// The k-means core over the m training rows T (HBM, m × d).  Centroids → cen_dev (nlist × d, HBM) and the
// final host copy cen_host; the last iteration's cluster sizes → sizes (optional).
// spherical k-means: every centroid renormalised to unit L2 norm (FAISS Clustering::post_process_centroids; fp64
// sum of squares, as oracle_kmeans_train's km_renorm)
static void km_renorm(std::vector<float> &cen, int nlist, int d) {
    for (int c = 0; c < nlist; ++c) {
        float *a = cen.data() + (size_t)c * d;
        double s = 0.0;
        for (int e = 0; e < d; ++e) s = s + (double)a[e] * (double)a[e];
        if (s > 0.0) {
            const float inv = (float)(1.0 / std::sqrt(s));
            for (int e = 0; e < d; ++e) a[e] *= inv;
        }
    }
}

void kmeans_core(int d, int metric, int nlist, const float *T, int64_t m, int niter, uint64_t rs, int init,
                 float *cen_dev, std::vector<float> &cen_host, int64_t *sizes, int device, hipStream_t st) {
    DevBuf sc;
    // ---- init ----
    if (init == HIPANN_KMEANS_INIT_RANDOM) {
        std::vector<int64_t> perm((size_t)m);
        for (int64_t i = 0; i < m; ++i) perm[(size_t)i] = i;
        std::vector<int64_t> pick((size_t)nlist);
        for (int64_t i = 0; i < nlist; ++i) {
            const int64_t j = i + (int64_t)(km_next(rs) % (uint64_t)(m - i));
            std::swap(perm[(size_t)i], perm[(size_t)j]);
            pick[(size_t)i] = perm[(size_t)i];
        }
        DevBuf prow;
        prow.ensure(sizeof(int64_t) * (size_t)nlist, device);
        HIPANN_CHECK(hipMemcpyAsync(prow.p, pick.data(), sizeof(int64_t) * (size_t)nlist, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(km_gather, dim3((unsigned)ceil_div((int64_t)nlist * d, 256)), dim3(256), 0, st, T,
                           prow.get<int64_t>(), (int64_t)nlist, d, cen_dev);
        HIPANN_CHECK(hipGetLastError());
        HIPANN_CHECK(hipStreamSynchronize(st));
    } else {
        HIPANN_REQUIRE(init == HIPANN_KMEANS_INIT_PLUSPLUS, "ivf train: init must be 0 (random) or 1 (k-means++)");
        const int nb = (int)ceil_div(m, 256);
        DevBuf d2, mx, bsum;
        d2.ensure(sizeof(double) * (size_t)m, device);
        mx.ensure(sizeof(unsigned long long), device);
        bsum.ensure(sizeof(unsigned long long) * (size_t)nb, device);
        HIPANN_CHECK(hipMemsetAsync(mx.p, 0, sizeof(unsigned long long), st));
        hipLaunchKernelGGL(km_fill_d2, dim3((unsigned)nb), dim3(256), 0, st, d2.get<double>(), m);
        const int64_t first = (int64_t)(km_next(rs) % (uint64_t)m);
        HIPANN_CHECK(hipMemcpyAsync(cen_dev, T + first * (int64_t)d, sizeof(float) * (size_t)d,
                                    hipMemcpyDeviceToDevice, st));
        for (int j = 1; j < nlist; ++j) {
            hipLaunchKernelGGL(kpp_update, dim3((unsigned)ceil_div(m, 4)), dim3(256), 0, st, T, m, d,
                               cen_dev + (int64_t)(j - 1) * d, d2.get<double>(), mx.get<unsigned long long>());
            hipLaunchKernelGGL(kpp_weights, dim3((unsigned)nb), dim3(256), 0, st, d2.get<double>(), m,
                               mx.get<unsigned long long>(), bsum.get<unsigned long long>());
            hipLaunchKernelGGL(kpp_pick, dim3(1), dim3(256), 0, st, d2.get<double>(), m, mx.get<unsigned long long>(),
                               bsum.get<unsigned long long>(), nb, (unsigned long long)km_next(rs), T, d,
                               cen_dev + (int64_t)j * d);
        }
        HIPANN_CHECK(hipGetLastError());
        HIPANN_CHECK(hipStreamSynchronize(st));
    }
    cen_host.resize((size_t)nlist * d);
    HIPANN_CHECK(hipMemcpyAsync(cen_host.data(), cen_dev, sizeof(float) * cen_host.size(), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    if (metric == kIP) {  // FAISS post_process_centroids after the init: unit-norm centroids before the first assignment
        km_renorm(cen_host, nlist, d);
        HIPANN_CHECK(hipMemcpyAsync(cen_dev, cen_host.data(), sizeof(float) * cen_host.size(), hipMemcpyHostToDevice, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
    }
    if (niter <= 0) {
        if (sizes) std::fill(sizes, sizes + nlist, (int64_t)0);
        return;
    }
    // ---- Lloyd ----
    FlatIndex q;
    q.form = kFlatFp32;  // exact fp32 products, the coarse quantizer's form
    q.d = d;
    q.metric = metric;
    {
        auto sh = std::make_unique<FlatShard>();
        sh->device = device;
        sh->xb = cen_dev;
        sh->owns = false;
        sh->n = nlist;
        sh->cap = nlist;
        q.shards.push_back(std::move(sh));
    }
    FlatShard &qs = *q.shards[0];
    const int64_t bs = 65536;
    DevBuf Dd, Ii, key, val, key2, val2, cnt, off, S, tmp;
    Dd.ensure(sizeof(float) * (size_t)std::min(m, bs), device);
    Ii.ensure(sizeof(int64_t) * (size_t)m, device);
    key.ensure(sizeof(unsigned) * (size_t)m, device);
    val.ensure(sizeof(unsigned) * (size_t)m, device);
    key2.ensure(sizeof(unsigned) * (size_t)m, device);
    val2.ensure(sizeof(unsigned) * (size_t)m, device);
    cnt.ensure(sizeof(int) * (size_t)nlist, device);
    off.ensure(sizeof(int64_t) * (size_t)(nlist + 1), device);
    S.ensure(sizeof(double) * (size_t)nlist * d, device);
    size_t tmp_bytes = 0;
    int end_bit = 1;
    while ((1ll << end_bit) <= nlist) ++end_bit;  // keys 0..nlist
    HIPANN_CHECK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key.get<unsigned>(), key2.get<unsigned>(),
                                           val.get<unsigned>(), val2.get<unsigned>(), (size_t)m, 0, end_bit, st));
    tmp.ensure(std::max<size_t>(tmp_bytes, 256), device);
    std::vector<int> hcnt((size_t)nlist);
    std::vector<int64_t> hoff((size_t)nlist + 1);
    std::vector<double> hS((size_t)nlist * d);
    std::vector<float> hs((size_t)nlist);
    const float EPS = 1.f / 1024.f;
    for (int it = 0; it < niter; ++it) {
        if (metric == kL2) {
            qs.xn.ensure(sizeof(float) * (size_t)nlist, device);
            launch_row_norms(cen_dev, nlist, d, qs.xn.get<float>(), st);
        }
        for (int64_t r0 = 0; r0 < m; r0 += bs) {
            const int64_t mm = std::min(bs, m - r0);
            flat_shard_search(q, qs, mm, T + r0 * d, 1, 1, Dd.get<float>(), Ii.get<int64_t>() + r0, st);
        }
        HIPANN_CHECK(hipMemsetAsync(cnt.p, 0, sizeof(int) * (size_t)nlist, st));
        hipLaunchKernelGGL(km_keys, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, st, Ii.get<int64_t>(), m, nlist,
                           key.get<unsigned>(), val.get<unsigned>(), cnt.get<int>());
        HIPANN_CHECK(hipGetLastError());
        size_t tb = tmp.bytes;
        HIPANN_CHECK(rocprim::radix_sort_pairs(tmp.p, tb, key.get<unsigned>(), key2.get<unsigned>(), val.get<unsigned>(),
                                               val2.get<unsigned>(), (size_t)m, 0, end_bit, st));
        HIPANN_CHECK(hipMemcpyAsync(hcnt.data(), cnt.p, sizeof(int) * (size_t)nlist, hipMemcpyDeviceToHost, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
        hoff[0] = 0;
        for (int c = 0; c < nlist; ++c) hoff[(size_t)c + 1] = hoff[(size_t)c] + hcnt[(size_t)c];
        HIPANN_CHECK(hipMemcpyAsync(off.p, hoff.data(), sizeof(int64_t) * hoff.size(), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(km_sums, dim3((unsigned)nlist), dim3(256), 0, st, T, d, val2.get<unsigned>(),
                           off.get<int64_t>(), S.get<double>());
        HIPANN_CHECK(hipGetLastError());
        HIPANN_CHECK(hipMemcpyAsync(hS.data(), S.p, sizeof(double) * hS.size(), hipMemcpyDeviceToHost, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
        // means, FAISS's split_clusters (float cluster sizes, halved exactly), spherical renorm (IP)
        for (int c = 0; c < nlist; ++c) {
            if (!hcnt[(size_t)c]) continue;
            for (int e = 0; e < d; ++e)
                cen_host[(size_t)c * d + e] = (float)(hS[(size_t)c * d + e] / (double)hcnt[(size_t)c]);
        }
        for (int c = 0; c < nlist; ++c) hs[(size_t)c] = (float)hcnt[(size_t)c];
        for (int ci = 0; ci < nlist; ++ci) {
            if (hs[(size_t)ci] != 0.f) continue;
            int cj = 0;
            for (;; cj = (cj + 1) % nlist) {
                const float p = (float)(((double)hs[(size_t)cj] - 1.0) / (double)(float)(m - nlist));
                const float r = km_rand_float(rs);
                if (r < p) break;
            }
            float *a = cen_host.data() + (size_t)ci * d, *b = cen_host.data() + (size_t)cj * d;
            std::memcpy(a, b, sizeof(float) * (size_t)d);
            for (int e = 0; e < d; ++e) {
                if (e % 2 == 0) { a[e] *= 1 + EPS; b[e] *= 1 - EPS; }
                else { a[e] *= 1 - EPS; b[e] *= 1 + EPS; }
            }
            hs[(size_t)ci] = hs[(size_t)cj] / 2;
            hs[(size_t)cj] -= hs[(size_t)ci];
        }
        if (metric == kIP) km_renorm(cen_host, nlist, d);  // spherical
        HIPANN_CHECK(hipMemcpyAsync(cen_dev, cen_host.data(), sizeof(float) * cen_host.size(), hipMemcpyHostToDevice, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
    }
    if (sizes)
        for (int c = 0; c < nlist; ++c) sizes[c] = hcnt[(size_t)c];
}

void check_train_args(int d, int metric, int nlist, int64_t n, int niter) {
    HIPANN_REQUIRE(d > 0 && nlist > 0 && n > 0, "ivf train: d, nlist and n must be > 0");
    HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 (L2) or 1 (IP)");
    HIPANN_REQUIRE(niter >= 0, "ivf train: niter must be >= 0");
    HIPANN_REQUIRE((int64_t)256 * nlist < (int64_t)0x7fffffff, "ivf train: nlist too large");
}

void set_err(char *buf, int len, const char *msg) {
    if (!buf || len <= 0) return;
    std::strncpy(buf, msg, (size_t)len - 1);
    buf[len - 1] = '\0';
}

template <typename F>
int guard(char *eb, int el, F &&f) {
    try {
        return f();
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

struct TrainStream {
    hipStream_t s = nullptr;
    int dev;
    explicit TrainStream(int d) : dev(d) {
        DeviceGuard g(d);
        HIPANN_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    ~TrainStream() {
        DeviceGuard g(dev);
        (void)hipStreamDestroy(s);
    }
};

}  // namespace
}  // namespace hipann

using namespace hipann;

extern "C" {

int hipann_ivf_train(int d, int metric, int nlist, int64_t n, const float *x, int64_t train_sample, int niter,
                     uint64_t seed, int init, int device, float *centroids, int64_t *list_sizes, char *eb, int el) {
    return guard(eb, el, [&]() -> int {
        check_train_args(d, metric, nlist, n, niter);
        HIPANN_REQUIRE(x && centroids, "ivf train: null buffer");
        int ndev = 0;
        HIPANN_REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0, "no HIP device");
        HIPANN_REQUIRE(device >= 0 && device < ndev, "invalid device");
        DeviceGuard g(device);
        TrainStream ts(device);
        uint64_t rs = seed;
        const std::vector<int64_t> rows = training_rows(n, train_sample, nlist, rs);
        const int64_t m = (int64_t)rows.size();
        // only the training rows travel: gathered on the host (the extension holds all_vectors in host memory)
        HostBuf h;
        h.ensure(sizeof(float) * (size_t)m * d);
        for (int64_t i = 0; i < m; ++i)
            std::memcpy(h.get<float>() + i * d, x + rows[(size_t)i] * d, sizeof(float) * (size_t)d);
        DevBuf T, cen;
        T.ensure(sizeof(float) * (size_t)m * d, device);
        cen.ensure(sizeof(float) * (size_t)nlist * d, device);
        HIPANN_CHECK(hipMemcpyAsync(T.p, h.p, sizeof(float) * (size_t)m * d, hipMemcpyHostToDevice, ts.s));
        std::vector<float> out;
        kmeans_core(d, metric, nlist, T.get<float>(), m, niter, rs, init, cen.get<float>(), out, list_sizes, device, ts.s);
        std::memcpy(centroids, out.data(), sizeof(float) * out.size());
        return 0;
    });
}

int hipann_ivf_train_device(int d, int metric, int nlist, int64_t n, const float *x_dev, int64_t train_sample,
                            int niter, uint64_t seed, int init, int device, float *centroids_dev, void *stream,
                            char *eb, int el) {
    return guard(eb, el, [&]() -> int {
        check_train_args(d, metric, nlist, n, niter);
        HIPANN_REQUIRE(x_dev && centroids_dev, "ivf train: null buffer");
        int ndev = 0;
        HIPANN_REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0, "no HIP device");
        HIPANN_REQUIRE(device >= 0 && device < ndev, "invalid device");
        DeviceGuard g(device);
        hipStream_t st = static_cast<hipStream_t>(stream);
        uint64_t rs = seed;
        const std::vector<int64_t> rows = training_rows(n, train_sample, nlist, rs);
        const int64_t m = (int64_t)rows.size();
        DevBuf T, drows;
        T.ensure(sizeof(float) * (size_t)m * d, device);
        drows.ensure(sizeof(int64_t) * (size_t)m, device);
        HIPANN_CHECK(hipMemcpyAsync(drows.p, rows.data(), sizeof(int64_t) * (size_t)m, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(km_gather, dim3((unsigned)ceil_div(m * d, 256)), dim3(256), 0, st, x_dev,
                           drows.get<int64_t>(), m, d, T.get<float>());
        HIPANN_CHECK(hipGetLastError());
        std::vector<float> out;
        kmeans_core(d, metric, nlist, T.get<float>(), m, niter, rs, init, centroids_dev, out, nullptr, device, st);
        return 0;
    });
}

}  // extern "C"
