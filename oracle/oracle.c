/*
 * oracle.c — CPU restatement of the reference's search semantics.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline.  The product (libhipann.so) never links or calls it.
 *
 * What is restated (the reference cannot be built here: FAISS 1.13.2, DuckDB and the Rust crates are
 * absent; see DESIGN.md "Oracle"):
 *
 *  FAISS 1.13.2 CPU (external dependency pinned in the reference at vcpkg.json:3, FIXES.md:3), as
 *  called by the extension (src/faiss_index.cpp:737) and by faiss-metal's tests
 *  (faiss-metal/tests/test_metal_flat.mm:24-60):
 *   - IndexFlat{L2,IP}::search → knn_L2sqr / knn_inner_product:
 *       nq <  distance_compute_blas_threshold (20): direct fvec_L2sqr / fvec_inner_product per pair;
 *       nq >= 20: x_norms + y_norms − 2·ip over 4096×1024 (query × database) blocks, clamped ≥ 0.
 *     Result handler: max-heap (CMax) for L2 / min-heap (CMin) for IP with FAISS's strict admission
 *     (C::cmp(top, dis)), cmp2 id tie-break while sifting, heap_reorder at the end.
 *     Unfilled slots: (C::neutral() = ±FLT_MAX, −1).
 *   - IndexIVFFlat::search: quantizer->search(nq, x, nprobe) with the Flat rules above, then every
 *     probed list scanned in probe order with direct distances into one heap per query.
 *  rust_lib (the extension's DiskANN path):
 *   - distance.rs:15-24 (L2 = squared Euclidean, IP = −dot);  ann_search.cpp:702-720
 *     (ComputeDistancesCPU: sequential float sum, the reference CPU fallback of the bridge);
 *   - SQ8 codec provider.rs:161-210 (encode) and :140-146 (decode);
 *   - DiskProvider::search_batch lock-step BFS (disk_provider.rs:470-652) with insert_result
 *     (:656-678) and Rust's slice::binary_search_by (std 1.82+ form) for the insertion point.
 *
 * Floating point: compiled with -ffp-contract=off; every sum is sequential fp32 unless noted, and a
 * parallel fp64 "exact" distance is exported for the tests' near-tie windows.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_L2 0
#define ORACLE_IP 1

/* ------------------------------------------------------------------------------------------ */
/* distances                                                                                  */
/* ------------------------------------------------------------------------------------------ */

/* Summation order: SIMD-reduced like FAISS's fvec_L2sqr / fvec_inner_product (8-lane partial sums
 * under AVX2); fp32 throughout. */
static float l2sqr_f32(const float *a, const float *b, int d) {
    float s = 0.f;
#pragma omp simd reduction(+ : s)
    for (int j = 0; j < d; ++j) {
        const float t = a[j] - b[j];
        s += t * t;
    }
    return s;
}

static float dot_f32(const float *a, const float *b, int d) {
    float s = 0.f;
#pragma omp simd reduction(+ : s)
    for (int j = 0; j < d; ++j) s += a[j] * b[j];
    return s;
}

static float norm_f32(const float *a, int d) { return dot_f32(a, a, d); }

double oracle_exact_l2(const float *a, const float *b, int d) {
    double s = 0.0;
    for (int j = 0; j < d; ++j) {
        const double t = (double)a[j] - (double)b[j];
        s += t * t;
    }
    return s;
}

double oracle_exact_ip(const float *a, const float *b, int d) {
    double s = 0.0;
    for (int j = 0; j < d; ++j) s += (double)a[j] * (double)b[j];
    return s;
}

/* exact (fp64) distance of query q to each of m labelled rows (labels < 0 → NAN) */
void oracle_exact_dists(const float *xb, int d, const float *q, const int64_t *labels, int64_t m, int metric,
                        double *out) {
    for (int64_t i = 0; i < m; ++i) {
        if (labels[i] < 0) { out[i] = NAN; continue; }
        const float *x = xb + labels[i] * (int64_t)d;
        out[i] = metric == ORACLE_L2 ? oracle_exact_l2(q, x, d) : oracle_exact_ip(q, x, d);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* FAISS heaps (faiss/utils/Heap.h) — is_max = 1 for CMax (L2), 0 for CMin (IP)              */
/* ------------------------------------------------------------------------------------------ */

static int cmp1(int is_max, float a, float b) { return is_max ? a > b : a < b; }
static int cmp2(int is_max, float a1, float b1, int64_t a2, int64_t b2) {
    return is_max ? ((a1 > b1) || ((a1 == b1) && (a2 > b2))) : ((a1 < b1) || ((a1 == b1) && (a2 > b2)));
}
static float neutral(int is_max) { return is_max ? FLT_MAX : -FLT_MAX; }

static void heap_heapify(int is_max, size_t k, float *v, int64_t *ids) {
    for (size_t i = 0; i < k; ++i) { v[i] = neutral(is_max); ids[i] = -1; }
}

static void heap_replace_top(int is_max, size_t k, float *bv, int64_t *bi, float val, int64_t id) {
    bv--; bi--;
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k) break;
        if ((i2 == k + 1) || cmp2(is_max, bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2(is_max, val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1]; bi[i] = bi[i1]; i = i1;
        } else {
            if (cmp2(is_max, val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2]; bi[i] = bi[i2]; i = i2;
        }
    }
    bv[i] = val;
    bi[i] = id;
}

static void heap_pop(int is_max, size_t k, float *bv, int64_t *bi) {
    bv--; bi--;
    const float val = bv[k];
    const int64_t id = bi[k];
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k) break;
        if ((i2 == k + 1) || cmp2(is_max, bv[i1], bv[i2], bi[i1], bi[i2])) {
            if (cmp2(is_max, val, bv[i1], id, bi[i1])) break;
            bv[i] = bv[i1]; bi[i] = bi[i1]; i = i1;
        } else {
            if (cmp2(is_max, val, bv[i2], id, bi[i2])) break;
            bv[i] = bv[i2]; bi[i] = bi[i2]; i = i2;
        }
    }
    bv[i] = bv[k];
    bi[i] = bi[k];
}

static void heap_reorder(int is_max, size_t k, float *bv, int64_t *bi) {
    size_t i, ii;
    for (i = 0, ii = 0; i < k; i++) {
        const float val = bv[0];
        const int64_t id = bi[0];
        heap_pop(is_max, k - i, bv, bi);
        bv[k - ii - 1] = val;
        bi[k - ii - 1] = id;
        if (id != -1) ii++;
    }
    memmove(bv, bv + k - ii, ii * sizeof(*bv));
    memmove(bi, bi + k - ii, ii * sizeof(*bi));
    for (; ii < k; ii++) { bv[ii] = neutral(is_max); bi[ii] = -1; }
}

/* offer one candidate: FAISS result handlers admit when C::cmp(top, dis) (strict) */
static void heap_offer(int is_max, size_t k, float *bv, int64_t *bi, float dis, int64_t id) {
    if (cmp1(is_max, bv[0], dis)) heap_replace_top(is_max, k, bv, bi, dis, id);
}

/* ------------------------------------------------------------------------------------------ */
/* IndexFlat::search                                                                         */
/* ------------------------------------------------------------------------------------------ */

#define BLAS_THRESHOLD 20
#define BLAS_QUERY_BS 4096
#define BLAS_DB_BS 1024

/* D/I: nq*k.  Labels are label_offset + row. */
void oracle_flat_search(const float *xb, int64_t n, int d, const float *xq, int64_t nq, int k, int metric,
                        int64_t label_offset, float *D, int64_t *I) {
    const int is_max = metric == ORACLE_L2;
    if (nq < BLAS_THRESHOLD) {
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t i = 0; i < nq; ++i) {
            float *bv = D + i * k;
            int64_t *bi = I + i * k;
            heap_heapify(is_max, k, bv, bi);
            const float *q = xq + i * (int64_t)d;
            for (int64_t j = 0; j < n; ++j) {
                const float *x = xb + j * (int64_t)d;
                const float dis = metric == ORACLE_L2 ? l2sqr_f32(q, x, d) : dot_f32(q, x, d);
                heap_offer(is_max, k, bv, bi, dis, label_offset + j);
            }
            heap_reorder(is_max, k, bv, bi);
        }
        return;
    }
    /* BLAS path (exhaustive_L2sqr_blas / exhaustive_inner_product_blas) */
    float *xn = NULL, *yn = NULL;
    if (metric == ORACLE_L2) {
        xn = (float *)malloc(sizeof(float) * (size_t)nq);
        yn = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
#pragma omp parallel for
        for (int64_t i = 0; i < nq; ++i) xn[i] = norm_f32(xq + i * (int64_t)d, d);
#pragma omp parallel for
        for (int64_t j = 0; j < n; ++j) yn[j] = norm_f32(xb + j * (int64_t)d, d);
    }
    for (int64_t i = 0; i < nq; ++i) heap_heapify(is_max, k, D + i * k, I + i * k);
    for (int64_t i0 = 0; i0 < nq; i0 += BLAS_QUERY_BS) {
        const int64_t i1 = i0 + BLAS_QUERY_BS < nq ? i0 + BLAS_QUERY_BS : nq;
        for (int64_t j0 = 0; j0 < n; j0 += BLAS_DB_BS) {
            const int64_t j1 = j0 + BLAS_DB_BS < n ? j0 + BLAS_DB_BS : n;
#pragma omp parallel for schedule(dynamic, 4)
            for (int64_t i = i0; i < i1; ++i) {
                const float *q = xq + i * (int64_t)d;
                float *bv = D + i * k;
                int64_t *bi = I + i * k;
                for (int64_t j = j0; j < j1; ++j) {
                    const float ip = dot_f32(q, xb + j * (int64_t)d, d);
                    float dis;
                    if (metric == ORACLE_L2) {
                        dis = xn[i] + yn[j] - 2 * ip;
                        if (dis < 0) dis = 0;
                    } else {
                        dis = ip;
                    }
                    heap_offer(is_max, k, bv, bi, dis, label_offset + j);
                }
            }
        }
    }
    for (int64_t i = 0; i < nq; ++i) heap_reorder(is_max, k, D + i * k, I + i * k);
    free(xn);
    free(yn);
}

/* ------------------------------------------------------------------------------------------ */
/* IndexIVFFlat::search                                                                       */
/* ------------------------------------------------------------------------------------------ */

/* IndexIVF::search_preassigned (FAISS 1.13.2, external; called by IndexIVF::search after the coarse step):
 * the probe lists ci (nq*nprobe, probe order, -1 = skipped) are given; each query's lists are scanned in probe
 * order with the direct-form distance and offered to its heap (strict admission, cmp2 eviction). */
void oracle_ivf_search_preassigned(const int64_t *list_off, const int64_t *ids, const float *codes, int d,
                                   const float *xq, int64_t nq, int k, int nprobe, const int64_t *ci, int metric,
                                   float *D, int64_t *I) {
    const int is_max = metric == ORACLE_L2;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t i = 0; i < nq; ++i) {
        float *bv = D + i * k;
        int64_t *bi = I + i * k;
        heap_heapify(is_max, k, bv, bi);
        const float *q = xq + i * (int64_t)d;
        for (int p = 0; p < nprobe; ++p) {
            const int64_t l = ci[i * nprobe + p];
            if (l < 0) continue;
            for (int64_t r = list_off[l]; r < list_off[l + 1]; ++r) {
                const float *x = codes + r * (int64_t)d;
                const float dis = metric == ORACLE_L2 ? l2sqr_f32(q, x, d) : dot_f32(q, x, d);
                heap_offer(is_max, k, bv, bi, dis, ids[r]);
            }
        }
        heap_reorder(is_max, k, bv, bi);
    }
}

/* probes_out (nq*nprobe, may be NULL): coarse assignment in probe order. */
void oracle_ivf_search(const float *centroids, int nlist, const int64_t *list_off, const int64_t *ids,
                       const float *codes, int d, const float *xq, int64_t nq, int k, int nprobe, int metric, float *D,
                       int64_t *I, int64_t *probes_out) {
    const int is_max = metric == ORACLE_L2;
    if (nprobe > nlist) nprobe = nlist;
    float *cd = (float *)malloc(sizeof(float) * (size_t)nq * nprobe);
    int64_t *ci = (int64_t *)malloc(sizeof(int64_t) * (size_t)nq * nprobe);
    oracle_flat_search(centroids, nlist, d, xq, nq, nprobe, metric, 0, cd, ci);
    if (probes_out) memcpy(probes_out, ci, sizeof(int64_t) * (size_t)nq * nprobe);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t i = 0; i < nq; ++i) {
        float *bv = D + i * k;
        int64_t *bi = I + i * k;
        heap_heapify(is_max, k, bv, bi);
        const float *q = xq + i * (int64_t)d;
        for (int p = 0; p < nprobe; ++p) {
            const int64_t l = ci[i * nprobe + p];
            if (l < 0) continue;
            for (int64_t r = list_off[l]; r < list_off[l + 1]; ++r) {
                const float *x = codes + r * (int64_t)d;
                const float dis = metric == ORACLE_L2 ? l2sqr_f32(q, x, d) : dot_f32(q, x, d);
                heap_offer(is_max, k, bv, bi, dis, ids[r]);
            }
        }
        heap_reorder(is_max, k, bv, bi);
    }
    free(cd);
    free(ci);
}

/* ------------------------------------------------------------------------------------------ */
/* DiskANN distances (ann_search.cpp:702-720 ComputeDistancesCPU; distance.rs:15-24)          */
/* ------------------------------------------------------------------------------------------ */

static float diskann_dist(const float *q, const float *c, int d, int metric) {
    float s = 0.f;
    if (metric == ORACLE_L2) {
        for (int j = 0; j < d; ++j) {
            const float t = q[j] - c[j];
            s += t * t;
        }
    } else {
        for (int j = 0; j < d; ++j) s += q[j] * c[j];
        s = -s;
    }
    return s;
}

void oracle_batch_distances(const float *query, const float *cands, int n, int d, int metric, float *out) {
    for (int i = 0; i < n; ++i) out[i] = diskann_dist(query, cands + (int64_t)i * d, d, metric);
}

/* Timing model of the Rust caller's CPU distances (distance.rs:15-24 → diskann-vector 0.45's SIMD
 * SquaredL2 / InnerProduct, external): 16 independent fp32 accumulators (two 8-wide AVX2 vectors),
 * summed at the end.  Used only by bench.py to place MIN_GPU_WORK (metal_ffi.rs:36-46) against a
 * SIMD CPU; its rounding differs from the sequential sum, so no parity test uses it. */
void oracle_batch_distances_simd(const float *query, const float *cands, int n, int d, int metric, float *out) {
    for (int i = 0; i < n; ++i) {
        const float *c = cands + (int64_t)i * d;
        float acc[16] = {0};
        int j = 0;
        for (; j + 16 <= d; j += 16)
            for (int l = 0; l < 16; ++l) {
                const float t = metric == 1 ? query[j + l] * c[j + l] : (query[j + l] - c[j + l]) * (query[j + l] - c[j + l]);
                acc[l] += t;
            }
        float s = 0.f;
        for (int l = 0; l < 16; ++l) s += acc[l];
        for (; j < d; ++j) s += metric == 1 ? query[j] * c[j] : (query[j] - c[j]) * (query[j] - c[j]);
        out[i] = metric == 1 ? -s : s;
    }
}

void oracle_multi_batch_distances(const float *queries, const float *cands, const uint32_t *qmap, int total_n,
                                  int d, int metric, float *out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < total_n; ++i)
        out[i] = diskann_dist(queries + (int64_t)qmap[i] * d, cands + (int64_t)i * d, d, metric);
}

/* ------------------------------------------------------------------------------------------ */
/* SQ8 codec (provider.rs:161-210 quantize_sq8; :140-146 dequantize)                          */
/* ------------------------------------------------------------------------------------------ */

void oracle_sq8_train(const float *x, int64_t n, int d, float *mins, float *scale) {
    for (int j = 0; j < d; ++j) { mins[j] = FLT_MAX; scale[j] = -FLT_MAX; /* maxs */ }
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < d; ++j) {
            const float v = x[i * d + j];
            if (v < mins[j]) mins[j] = v;
            if (v > scale[j]) scale[j] = v;
        }
    for (int j = 0; j < d; ++j) {
        const float range = scale[j] - mins[j];
        scale[j] = range > 0.f ? range : 1.f;
    }
}

void oracle_sq8_encode(const float *x, int64_t n, int d, const float *mins, const float *scale, uint8_t *codes) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < d; ++j) {
            const float normalized = (x[i * d + j] - mins[j]) / scale[j];
            float v = roundf(normalized * 255.0f); /* f32::round: half away from zero */
            if (v < 0.f) v = 0.f;
            if (v > 255.f) v = 255.f;
            codes[i * d + j] = (uint8_t)v;
        }
}

void oracle_sq8_decode(const uint8_t *codes, int64_t n, int d, const float *mins, const float *scale, float *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < d; ++j) {
            const float a = (float)codes[i * d + j] / 255.0f;
            const float b = a * scale[j];
            out[i * d + j] = b + mins[j];
        }
}

/* distance of a query to an SQ8-coded row (dequantise, then the distance.rs formula) */
static float sq8_dist(const float *q, const uint8_t *code, const float *mins, const float *scale, int d, int metric) {
    float s = 0.f;
    for (int j = 0; j < d; ++j) {
        const float a = (float)code[j] / 255.0f;
        const float v = a * scale[j];
        const float x = v + mins[j];
        if (metric == ORACLE_L2) {
            const float t = q[j] - x;
            s += t * t;
        } else {
            s += q[j] * x;
        }
    }
    return metric == ORACLE_L2 ? s : -s;
}

void oracle_sq8_distances_ids(const float *queries, const uint8_t *codes, const float *mins, const float *scale,
                              int d, const uint32_t *ids, const uint32_t *qmap, int total_n, int metric, float *out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < total_n; ++i)
        out[i] = sq8_dist(queries + (int64_t)qmap[i] * d, codes + (int64_t)ids[i] * d, mins, scale, d, metric);
}

/* ------------------------------------------------------------------------------------------ */
/* DiskProvider::search_batch (disk_provider.rs:470-652) — lock-step best-first BFS             */
/* ------------------------------------------------------------------------------------------ */

typedef struct { float d; uint32_t id; } Cand;

/* min-heap on (d, id) — BinaryHeap<Reverse<(FloatOrd, u32)>> pops the smallest (d, id) */
typedef struct { Cand *a; size_t n, cap; } MinHeap;

static int cand_less(Cand x, Cand y) { return x.d < y.d || (x.d == y.d && x.id < y.id); }

static void mh_push(MinHeap *h, Cand c) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 64;
        h->a = (Cand *)realloc(h->a, h->cap * sizeof(Cand));
    }
    size_t i = h->n++;
    while (i > 0) {
        size_t p = (i - 1) / 2;
        if (!cand_less(c, h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = c;
}

static int mh_pop(MinHeap *h, Cand *out) {
    if (!h->n) return 0;
    *out = h->a[0];
    Cand last = h->a[--h->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        Cand best = last;
        if (l < h->n && cand_less(h->a[l], best)) { m = l; best = h->a[l]; }
        if (r < h->n && cand_less(h->a[r], best)) { m = r; }
        if (m == i) break;
        h->a[i] = h->a[m];
        i = m;
    }
    if (h->n) h->a[i] = last;
    return 1;
}

/* open-addressing u32 set */
typedef struct { uint32_t *slots; size_t cap, n; } USet;
#define USET_EMPTY 0xffffffffu
static void us_init(USet *s, size_t cap) {
    size_t c = 64;
    while (c < cap * 2) c <<= 1;
    s->slots = (uint32_t *)malloc(c * sizeof(uint32_t));
    memset(s->slots, 0xff, c * sizeof(uint32_t));
    s->cap = c;
    s->n = 0;
}
static int us_insert(USet *s, uint32_t v); /* fwd */
static void us_grow(USet *s) {
    uint32_t *old = s->slots;
    size_t oc = s->cap;
    s->cap *= 2;
    s->slots = (uint32_t *)malloc(s->cap * sizeof(uint32_t));
    memset(s->slots, 0xff, s->cap * sizeof(uint32_t));
    s->n = 0;
    for (size_t i = 0; i < oc; ++i)
        if (old[i] != USET_EMPTY) us_insert(s, old[i]);
    free(old);
}
/* returns 1 if newly inserted (HashSet::insert) */
static int us_insert(USet *s, uint32_t v) {
    if ((s->n + 1) * 2 > s->cap) us_grow(s);
    size_t m = s->cap - 1, i = ((size_t)v * 0x9E3779B97F4A7C15ull >> 17) & m;
    while (s->slots[i] != USET_EMPTY) {
        if (s->slots[i] == v) return 0;
        i = (i + 1) & m;
    }
    s->slots[i] = v;
    s->n++;
    return 1;
}

/* Rust slice::binary_search_by (std ≥ 1.82) over result[0..len) with partial_cmp(probe.d, dist),
 * NaN → Equal; returns Ok(pos) or Err(pos) — either way the insert position. */
static size_t rust_binary_search(const Cand *res, size_t len, float dist) {
    if (len == 0) return 0;
    size_t size = len, base = 0;
    while (size > 1) {
        const size_t half = size / 2, mid = base + half;
        const float p = res[mid].d;
        const int greater = p > dist; /* cmp == Greater */
        base = greater ? base : mid;
        size -= half;
    }
    const float p = res[base].d;
    const int less = p < dist, greater = p > dist;
    if (!less && !greater) return base;      /* Equal → Ok(base) */
    return base + (less ? 1 : 0);            /* Err */
}

typedef struct {
    USet visited;
    MinHeap cands;
    Cand *result;
    size_t rlen;
    int active;
} QState;

/* insert_result (disk_provider.rs:656-678) */
static void insert_result(QState *s, size_t l, float dist, uint32_t nb) {
    if (s->rlen < l || dist < s->result[s->rlen - 1].d) {
        const size_t pos = rust_binary_search(s->result, s->rlen, dist);
        memmove(s->result + pos + 1, s->result + pos, (s->rlen - pos) * sizeof(Cand));
        s->result[pos].d = dist;
        s->result[pos].id = nb;
        s->rlen++;
        if (s->rlen > l) s->rlen = l;
        Cand c = {dist, nb};
        mh_push(&s->cands, c);
    }
}

/* Vector access: fp32 rows (vecs) or SQ8 codes (codes + mins/scale; dequantised as provider.rs).
 * adjacency: N*R u32 with u32::MAX padding (file_format.rs:3-18); get_neighbors trims at the first
 * sentinel (disk_provider.rs:317-332).  Output: per query the first k (id, dist) of `result`, with
 * (u32::MAX → id −1, FLT_MAX) for missing slots (ffi.rs:759-762 convention).
 * stats_out[0] = distance evaluations, [1] = BFS steps (lock-step iterations). */
void oracle_diskann_search_batch(const float *vecs, const uint8_t *codes, const float *mins, const float *scale,
                                 uint32_t N, int d, const uint32_t *adj, int R, const uint32_t *eps, int n_ep,
                                 const float *queries, int nq, int k, int l_search, int metric, int64_t *out_ids,
                                 float *out_d, int64_t *stats_out) {
    if (k > (int)N) k = (int)N;
    const size_t l = (size_t)(l_search > k ? l_search : k);
    QState *st = (QState *)calloc((size_t)nq, sizeof(QState));
    int64_t nevals = 0, nsteps = 0;
#define DIST(qi, id)                                                                                       \
    (codes ? sq8_dist(queries + (int64_t)(qi) * d, codes + (int64_t)(id) * d, mins, scale, d, metric)      \
           : diskann_dist(queries + (int64_t)(qi) * d, vecs + (int64_t)(id) * d, d, metric))
    for (int qi = 0; qi < nq; ++qi) {
        QState *s = &st[qi];
        us_init(&s->visited, l * 2);
        s->result = (Cand *)malloc((l + 1) * sizeof(Cand));
        s->rlen = 0;
        s->active = 1;
        /* seed (disk_provider.rs:524-538): push to heap and result, then stable sort result */
        for (int e = 0; e < n_ep; ++e) {
            const uint32_t ep = eps[e];
            if (us_insert(&s->visited, ep)) {
                if (ep >= N) continue;
                const float dist = DIST(qi, ep);
                nevals++;
                Cand c = {dist, ep};
                mh_push(&s->cands, c);
                s->result[s->rlen++] = c;  /* n_ep is small (≤ l) */
            }
        }
        /* stable insertion sort by partial_cmp on distance */
        for (size_t i = 1; i < s->rlen; ++i) {
            Cand c = s->result[i];
            size_t j = i;
            while (j > 0 && s->result[j - 1].d > c.d) { s->result[j] = s->result[j - 1]; --j; }
            s->result[j] = c;
        }
    }
    uint32_t *nb_ids = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)nq * R + 1);
    uint32_t *nb_q = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)nq * R + 1);
    float *nb_d = (float *)malloc(sizeof(float) * (size_t)nq * R + 1);
    for (;;) {
        int active = 0;
        for (int qi = 0; qi < nq; ++qi) active += st[qi].active;
        if (!active) break;
        nsteps++;
        size_t tot = 0;
        for (int qi = 0; qi < nq; ++qi) {
            QState *s = &st[qi];
            if (!s->active) continue;
            Cand c;
            if (!mh_pop(&s->cands, &c)) { s->active = 0; continue; }
            if (s->rlen >= l && c.d > s->result[l - 1].d) { s->active = 0; continue; }
            const uint32_t *nbr = adj + (size_t)c.id * R;
            for (int r = 0; r < R; ++r) {
                const uint32_t nb = nbr[r];
                if (nb == 0xffffffffu) break;
                if (nb >= N) continue;
                if (!us_insert(&s->visited, nb)) continue;
                nb_ids[tot] = nb;
                nb_q[tot] = (uint32_t)qi;
                tot++;
            }
        }
        if (!tot) continue;
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < tot; ++i) nb_d[i] = DIST(nb_q[i], nb_ids[i]);
        nevals += (int64_t)tot;
        for (size_t i = 0; i < tot; ++i) insert_result(&st[nb_q[i]], l, nb_d[i], nb_ids[i]);
    }
#undef DIST
    for (int qi = 0; qi < nq; ++qi) {
        QState *s = &st[qi];
        for (int j = 0; j < k; ++j) {
            if ((size_t)j < s->rlen) {
                out_ids[(int64_t)qi * k + j] = s->result[j].id;
                out_d[(int64_t)qi * k + j] = s->result[j].d;
            } else {
                out_ids[(int64_t)qi * k + j] = -1;
                out_d[(int64_t)qi * k + j] = FLT_MAX;
            }
        }
        free(s->visited.slots);
        free(s->cands.a);
        free(s->result);
    }
    if (stats_out) { stats_out[0] = nevals; stats_out[1] = nsteps; }
    free(st);
    free(nb_ids);
    free(nb_q);
    free(nb_d);
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------------ */
/* IVF training (k-means): the restatement hipann_ivf_train is checked against                */
/* ------------------------------------------------------------------------------------------ */
/*
 * The extension trains its IndexIVFFlat on the CPU at CREATE INDEX (src/faiss_index.cpp:302-319: a
 * deterministic stride sample of train_sample rows, then faiss_idx->train → FAISS 1.13.2 IndexIVF::train_q1 →
 * Clustering::train, external).  hipann_ivf_train runs the same pipeline on the GPU; FAISS's own random draws
 * (its RandomGenerator over rand_perm / rand_float) are not reproduced, so the GPU is pinned to THIS
 * restatement, which fixes every draw to splitmix64(seed):
 *   1. training rows: the reference's stride sample (faiss_index.cpp:307-313) when 0 < train_sample < n;
 *   2. FAISS's max_points_per_centroid = 256: above 256·nlist rows, a uniform subset (partial Fisher-Yates,
 *      kept in ascending row order);
 *   3. init 0: FAISS's random init (the first nlist rows of a partial Fisher-Yates); init 1: k-means++ (D²
 *      sampling) with fp64 squared distances — each row's 64 lane-strided partial sums then an xor butterfly,
 *      the GPU kernel's order — and weights w = floor(d² · 2^32 / max d²) as integers, so the draw
 *      t = r mod Σw picks the same row whatever the summation order of the weights;
 *   4. niter Lloyd iterations (FAISS Clustering::train): assignment = the Flat search with k = 1 (this
 *      oracle's FAISS restatement: BLAS form at >= 20 rows), centroids = fp64 means in row order,
 *      FAISS's split_clusters for empty ones (EPS = 1/1024, split probability (n_j − 1)/(m − nlist)),
 *      and for IP the spherical renormalisation (IndexIVF sets cp.spherical for METRIC_INNER_PRODUCT) — after
 *      the init too (post_process_centroids runs before the first assignment).
 */
static uint64_t km_next(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static float km_rand_float(uint64_t *s) { return (float)(km_next(s) >> 40) * 0x1p-24f; }

/* squared L2 in fp64: 64 lane partials (lane l sums dims l, l+64, … in order), then the xor butterfly */
static double km_dist64(const float *a, const float *b, int d) {
    double p[64], t[64];
    for (int l = 0; l < 64; ++l) {
        double acc = 0.0;
        for (int e = l; e < d; e += 64) {
            const double df = (double)a[e] - (double)b[e];
            acc = acc + df * df;
        }
        p[l] = acc;
    }
    for (int o = 32; o > 0; o >>= 1) {
        for (int l = 0; l < 64; ++l) t[l] = p[l] + p[l ^ o];
        memcpy(p, t, sizeof p);
    }
    return p[0];
}

/* spherical k-means: every centroid renormalised to unit L2 norm (FAISS Clustering::post_process_centroids) */
static void km_renorm(float *centroids, int nlist, int d) {
    for (int c = 0; c < nlist; ++c) {
        float *a = centroids + (int64_t)c * d;
        double s = 0.0;
        for (int e = 0; e < d; ++e) s = s + (double)a[e] * (double)a[e];
        if (s > 0.0) {
            const float inv = (float)(1.0 / sqrt(s));
            for (int e = 0; e < d; ++e) a[e] *= inv;
        }
    }
}

int oracle_kmeans_train(const float *x, int64_t n, int d, int metric, int nlist, int64_t train_sample, int niter,
                        uint64_t seed, int init, float *centroids, int64_t *sizes_out) {
    if (d <= 0 || nlist <= 0 || n <= 0) return -1;
    uint64_t rs = seed;
    /* 1. stride sample */
    int64_t m = n;
    int64_t *rows = NULL;
    if (train_sample > 0 && train_sample < n) {
        m = train_sample;
        rows = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
        const double stride = (double)n / (double)train_sample;
        for (int64_t i = 0; i < m; ++i) rows[i] = (int64_t)((double)i * stride);
    } else {
        rows = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
        for (int64_t i = 0; i < m; ++i) rows[i] = i;
    }
    if (m < nlist) { free(rows); return -1; }
    /* 2. at most 256 per centroid */
    const int64_t maxp = (int64_t)256 * nlist;
    if (m > maxp) {
        int64_t *perm = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
        for (int64_t i = 0; i < m; ++i) perm[i] = i;
        for (int64_t i = 0; i < maxp; ++i) {
            const int64_t j = i + (int64_t)(km_next(&rs) % (uint64_t)(m - i));
            const int64_t tmp = perm[i]; perm[i] = perm[j]; perm[j] = tmp;
        }
        /* ascending row order: mark the chosen, then collect */
        char *pick = (char *)calloc((size_t)m, 1);
        for (int64_t i = 0; i < maxp; ++i) pick[perm[i]] = 1;
        int64_t w = 0;
        for (int64_t i = 0; i < m; ++i)
            if (pick[i]) rows[w++] = rows[i];
        free(pick);
        free(perm);
        m = maxp;
    }
    float *T = (float *)malloc(sizeof(float) * (size_t)m * d);
    for (int64_t i = 0; i < m; ++i) memcpy(T + i * (int64_t)d, x + rows[i] * (int64_t)d, sizeof(float) * (size_t)d);
    free(rows);
    /* 3. init */
    if (init == 0) {
        int64_t *perm = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
        for (int64_t i = 0; i < m; ++i) perm[i] = i;
        for (int64_t i = 0; i < nlist; ++i) {
            const int64_t j = i + (int64_t)(km_next(&rs) % (uint64_t)(m - i));
            const int64_t tmp = perm[i]; perm[i] = perm[j]; perm[j] = tmp;
            memcpy(centroids + i * (int64_t)d, T + perm[i] * (int64_t)d, sizeof(float) * (size_t)d);
        }
        free(perm);
    } else {
        double *d2 = (double *)malloc(sizeof(double) * (size_t)m);
        uint64_t *wt = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)m);
        for (int64_t i = 0; i < m; ++i) d2[i] = DBL_MAX;
        int64_t pick = (int64_t)(km_next(&rs) % (uint64_t)m);
        memcpy(centroids, T + pick * (int64_t)d, sizeof(float) * (size_t)d);
        for (int j = 1; j < nlist; ++j) {
            const float *c = centroids + (int64_t)(j - 1) * d;
            double mx = 0.0;
#pragma omp parallel for reduction(max : mx)
            for (int64_t i = 0; i < m; ++i) {
                const double v = km_dist64(T + i * (int64_t)d, c, d);
                if (v < d2[i]) d2[i] = v;
                if (d2[i] > mx) mx = d2[i];
            }
            const uint64_t r = km_next(&rs);
            if (mx > 0.0) {
                const double scale = 4294967296.0 / mx;
                uint64_t tot = 0;
                for (int64_t i = 0; i < m; ++i) { wt[i] = (uint64_t)(d2[i] * scale); tot += wt[i]; }
                const uint64_t t = r % tot;
                uint64_t acc = 0;
                pick = m - 1;
                for (int64_t i = 0; i < m; ++i) {
                    acc += wt[i];
                    if (acc > t) { pick = i; break; }
                }
            } else {
                pick = (int64_t)(r % (uint64_t)m);
            }
            memcpy(centroids + (int64_t)j * d, T + pick * (int64_t)d, sizeof(float) * (size_t)d);
        }
        free(d2);
        free(wt);
    }
    /* FAISS Clustering::train_encoded calls post_process_centroids() right after the init as well as after every
     * iteration: with spherical (IP) the initial centroids are unit vectors before the first assignment */
    if (metric == ORACLE_IP) km_renorm(centroids, nlist, d);
    /* 4. Lloyd */
    float *D = (float *)malloc(sizeof(float) * (size_t)m);
    int64_t *I = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
    double *S = (double *)malloc(sizeof(double) * (size_t)nlist * d);
    int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * (size_t)nlist);
    float *hs = (float *)malloc(sizeof(float) * (size_t)nlist);
    const float EPS = 1.f / 1024.f;
    for (int it = 0; it < niter; ++it) {
        oracle_flat_search(centroids, nlist, d, T, m, 1, metric, 0, D, I);
        memset(S, 0, sizeof(double) * (size_t)nlist * d);
        memset(cnt, 0, sizeof(int64_t) * (size_t)nlist);
        for (int64_t i = 0; i < m; ++i) {
            const int64_t a = I[i];
            if (a < 0 || a >= nlist) continue;
            cnt[a]++;
            double *s = S + a * (int64_t)d;
            const float *xi = T + i * (int64_t)d;
            for (int e = 0; e < d; ++e) s[e] = s[e] + (double)xi[e];
        }
        for (int c = 0; c < nlist; ++c) {
            if (!cnt[c]) continue;
            for (int e = 0; e < d; ++e)
                centroids[(int64_t)c * d + e] = (float)(S[(int64_t)c * d + e] / (double)cnt[c]);
        }
        /* FAISS split_clusters (clustering.cpp): its cluster sizes are floats (hassign), halved exactly */
        for (int c = 0; c < nlist; ++c) hs[c] = (float)cnt[c];
        for (int ci = 0; ci < nlist; ++ci) {
            if (hs[ci] != 0.f) continue;
            int cj = 0;
            for (;; cj = (cj + 1) % nlist) {
                const float p = (float)(((double)hs[cj] - 1.0) / (double)(float)(m - nlist));
                const float r = km_rand_float(&rs);
                if (r < p) break;
            }
            float *a = centroids + (int64_t)ci * d, *b = centroids + (int64_t)cj * d;
            memcpy(a, b, sizeof(float) * (size_t)d);
            for (int e = 0; e < d; ++e) {
                if (e % 2 == 0) { a[e] *= 1 + EPS; b[e] *= 1 - EPS; }
                else { a[e] *= 1 - EPS; b[e] *= 1 + EPS; }
            }
            hs[ci] = hs[cj] / 2;
            hs[cj] -= hs[ci];
        }
        if (metric == ORACLE_IP) km_renorm(centroids, nlist, d); /* spherical */
    }
    if (sizes_out)
        for (int c = 0; c < nlist; ++c) sizes_out[c] = niter > 0 ? cnt[c] : 0;
    free(D);
    free(I);
    free(S);
    free(cnt);
    free(hs);
    free(T);
    return 0;
}
