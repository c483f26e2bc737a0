/* oracle_selftest.c — TEST PROGRAM (test infrastructure only, like oracle.c): drives every entry point of the CPU
 * oracle on small seeded inputs and checks the invariants the parity tests rely on, so that the oracle can be built
 * and run under AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle sanitize`, tests/test_sanitizers.py).
 * It is not a parity test: the oracle's answers are pinned against the reference's fixtures in tests/test_oracle.py.
 * Exit status 0 = every check passed; a sanitizer report aborts (-fno-sanitize-recover=all). */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* oracle.c's entry points (no header: the Python side binds them with ctypes) */
double oracle_exact_l2(const float *a, const float *b, int d);
double oracle_exact_ip(const float *a, const float *b, int d);
void oracle_exact_dists(const float *xb, int d, const float *q, const int64_t *labels, int64_t m, int metric,
                        double *out);
void oracle_flat_search(const float *xb, int64_t n, int d, const float *xq, int64_t nq, int k, int metric,
                        int64_t label_offset, float *D, int64_t *I);
void oracle_ivf_search_preassigned(const int64_t *list_off, const int64_t *ids, const float *codes, int d,
                                   const float *xq, int64_t nq, int k, int nprobe, const int64_t *ci, int metric,
                                   float *D, int64_t *I);
void oracle_ivf_search(const float *centroids, int nlist, const int64_t *list_off, const int64_t *ids,
                       const float *codes, int d, const float *xq, int64_t nq, int k, int nprobe, int metric, float *D,
                       int64_t *I, int64_t *probes_out);
void oracle_batch_distances(const float *query, const float *cands, int n, int d, int metric, float *out);
void oracle_batch_distances_simd(const float *query, const float *cands, int n, int d, int metric, float *out);
void oracle_multi_batch_distances(const float *queries, const float *cands, const uint32_t *qmap, int total_n,
                                  int d, int metric, float *out);
void oracle_sq8_train(const float *x, int64_t n, int d, float *mins, float *scale);
void oracle_sq8_encode(const float *x, int64_t n, int d, const float *mins, const float *scale, uint8_t *codes);
void oracle_sq8_decode(const uint8_t *codes, int64_t n, int d, const float *mins, const float *scale, float *out);
void oracle_sq8_distances_ids(const float *queries, const uint8_t *codes, const float *mins, const float *scale,
                              int d, const uint32_t *ids, const uint32_t *qmap, int total_n, int metric, float *out);
void oracle_diskann_search_batch(const float *vecs, const uint8_t *codes, const float *mins, const float *scale,
                                 uint32_t N, int d, const uint32_t *adj, int R, const uint32_t *eps, int n_ep,
                                 const float *queries, int nq, int k, int l_search, int metric, int64_t *out_ids,
                                 float *out_d, int64_t *stats_out);
int oracle_kmeans_train(const float *x, int64_t n, int d, int metric, int nlist, int64_t train_sample, int niter,
                        uint64_t seed, int init, float *centroids, int64_t *sizes_out);

static int failures = 0;
#define CHECK(c, ...)                                                                                  \
    do {                                                                                               \
        if (!(c)) {                                                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                                      \
            fprintf(stderr, __VA_ARGS__);                                                              \
            fprintf(stderr, "\n");                                                                     \
            ++failures;                                                                                \
        }                                                                                              \
    } while (0)

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static float urand(void) { /* splitmix64 → [-1, 1) */
    uint64_t z = (rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (float)((double)(z >> 11) / 9007199254740992.0 * 2.0 - 1.0);
}
static float *rand_mat(int64_t n, int d) {
    float *x = (float *)malloc(sizeof(float) * (size_t)(n * d > 0 ? n * d : 1));
    for (int64_t i = 0; i < n * d; ++i) x[i] = urand();
    return x;
}

/* exact brute force in double: the k smallest (key, row) — key = L2 distance or −IP */
static void brute(const float *xb, int64_t n, int d, const float *q, int metric, int k, int64_t *out) {
    double *key = (double *)malloc(sizeof(double) * (size_t)n);
    char *used = (char *)calloc((size_t)n, 1);
    for (int64_t j = 0; j < n; ++j)
        key[j] = metric == 0 ? oracle_exact_l2(q, xb + j * d, d) : -oracle_exact_ip(q, xb + j * d, d);
    for (int t = 0; t < k; ++t) {
        int64_t best = -1;
        for (int64_t j = 0; j < n; ++j)
            if (!used[j] && (best < 0 || key[j] < key[best])) best = j;
        out[t] = best;
        if (best >= 0) used[best] = 1;
    }
    free(key);
    free(used);
}

static void test_flat(void) {
    const int64_t n = 300;
    const int d = 24, k = 7;
    float *xb = rand_mat(n, d);
    for (int metric = 0; metric < 2; ++metric)
        for (int nq = 5; nq <= 25; nq += 20) { /* nq < 20: per-query heaps; nq ≥ 20: the BLAS-path blocks */
            float *xq = rand_mat(nq, d);
            float *D = (float *)malloc(sizeof(float) * (size_t)nq * k);
            int64_t *I = (int64_t *)malloc(sizeof(int64_t) * (size_t)nq * k);
            oracle_flat_search(xb, n, d, xq, nq, k, metric, 1000, D, I);
            for (int i = 0; i < nq; ++i) {
                int64_t ref[7];
                brute(xb, n, d, xq + i * d, metric, k, ref);
                CHECK(I[i * k] - 1000 == ref[0], "flat top-1 metric %d nq %d query %d: %lld vs %lld", metric, nq, i,
                      (long long)I[i * k], (long long)ref[0]);
                for (int t = 1; t < k; ++t)
                    CHECK(metric == 0 ? D[i * k + t - 1] <= D[i * k + t] : D[i * k + t - 1] >= D[i * k + t],
                          "flat order metric %d query %d slot %d", metric, i, t);
            }
            free(xq);
            free(D);
            free(I);
        }
    /* k > n: FAISS pads with (±inf / FLT_MAX, −1) */
    {
        float *xq = rand_mat(2, d);
        float D[2 * 10];
        int64_t I[2 * 10];
        oracle_flat_search(xb, 4, d, xq, 2, 10, 0, 0, D, I);
        CHECK(I[4] == -1 && I[9] == -1 && I[0] >= 0, "flat k > n padding");
        free(xq);
    }
    free(xb);
}

static void test_ivf(void) {
    const int64_t n = 400;
    const int d = 16, nlist = 8, k = 5, nq = 23;
    float *xb = rand_mat(n, d), *xq = rand_mat(nq, d);
    float cen[8 * 16];
    memcpy(cen, xb, sizeof(cen));
    /* lists: rows assigned to their nearest centroid (row order kept), list 7 left empty */
    int64_t *assign = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    float cd1[1];
    for (int64_t j = 0; j < n; ++j) {
        oracle_flat_search(cen, nlist - 1, d, xb + j * d, 1, 1, 0, 0, cd1, assign + j);
    }
    int64_t off[9] = {0};
    for (int64_t j = 0; j < n; ++j) off[assign[j] + 1]++;
    for (int l = 0; l < nlist; ++l) off[l + 1] += off[l];
    int64_t cur[8];
    memcpy(cur, off, sizeof(cur));
    int64_t *ids = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    float *codes = (float *)malloc(sizeof(float) * (size_t)n * d);
    for (int64_t j = 0; j < n; ++j) {
        const int64_t r = cur[assign[j]]++;
        ids[r] = 100000 + j;
        memcpy(codes + r * d, xb + j * d, sizeof(float) * d);
    }
    for (int metric = 0; metric < 2; ++metric) {
        float D[23 * 5], Df[23 * 5], D2[23 * 5];
        int64_t I[23 * 5], If[23 * 5], I2[23 * 5], P[23 * 8];
        /* every list probed: the IVF answer is the Flat answer over the same rows */
        oracle_ivf_search(cen, nlist, off, ids, codes, d, xq, nq, k, nlist, metric, D, I, P);
        oracle_flat_search(xb, n, d, xq, nq, k, metric, 100000, Df, If);
        for (int i = 0; i < nq * k; ++i) CHECK(I[i] == If[i], "ivf full probe == flat, metric %d slot %d", metric, i);
        /* search_preassigned on the coarse step's own lists reproduces search */
        oracle_ivf_search(cen, nlist, off, ids, codes, d, xq, nq, k, 3, metric, D, I, P);
        oracle_ivf_search_preassigned(off, ids, codes, d, xq, nq, k, 3, P, metric, D2, I2);
        for (int i = 0; i < nq * k; ++i) CHECK(I[i] == I2[i] && D[i] == D2[i], "preassigned slot %d", i);
        /* skipped probes (−1) */
        for (int i = 0; i < nq * 3; ++i) P[i] = i % 3 == 1 ? -1 : P[i];
        oracle_ivf_search_preassigned(off, ids, codes, d, xq, nq, k, 3, P, metric, D2, I2);
    }
    free(xb);
    free(xq);
    free(assign);
    free(ids);
    free(codes);
}

static void test_distances_and_sq8(void) {
    const int n = 77, d = 37;
    float *q = rand_mat(3, d), *c = rand_mat(n, d);
    float a[77], b[77], m[77];
    uint32_t qmap[77], ids[77];
    for (int metric = 0; metric < 2; ++metric) {
        oracle_batch_distances(q, c, n, d, metric, a);
        oracle_batch_distances_simd(q, c, n, d, metric, b);
        for (int i = 0; i < n; ++i) {
            CHECK(fabsf(a[i] - b[i]) <= 1e-4f * (1.f + fabsf(a[i])), "simd vs scalar %d", i);
            qmap[i] = (uint32_t)(i % 3);
            ids[i] = (uint32_t)((i * 7) % n);
        }
        oracle_multi_batch_distances(q, c, qmap, n, d, metric, m);
        CHECK(m[0] == a[0], "multi batch query 0");
    }
    float mins[37], scale[37];
    oracle_sq8_train(c, n, d, mins, scale);
    uint8_t *codes = (uint8_t *)malloc((size_t)n * d);
    float *dec = (float *)malloc(sizeof(float) * (size_t)n * d);
    oracle_sq8_encode(c, n, d, mins, scale, codes);
    oracle_sq8_decode(codes, n, d, mins, scale, dec);
    for (int i = 0; i < n * d; ++i)
        CHECK(fabsf(dec[i] - c[i]) <= scale[i % d] / 255.f * 0.5001f + 1e-6f, "sq8 round trip %d", i);
    for (int metric = 0; metric < 2; ++metric) oracle_sq8_distances_ids(q, codes, mins, scale, d, ids, qmap, n, metric, m);
    free(q);
    free(c);
    free(codes);
    free(dec);
}

static void test_diskann(void) {
    const uint32_t N = 600;
    const int d = 20, R = 8, nq = 9, k = 6, L = 24;
    float *x = rand_mat(N, d), *q = rand_mat(nq, d);
    uint32_t *adj = (uint32_t *)malloc(sizeof(uint32_t) * N * R);
    for (uint32_t i = 0; i < N; ++i)
        for (int r = 0; r < R; ++r) /* a ring plus pseudo-random chords; some rows end early (u32::MAX sentinel) */
            adj[i * R + r] = (r == R - 1 && i % 5 == 0) ? UINT32_MAX : (r < 2 ? (i + 1 + r) % N : (uint32_t)((i * 131u + 17u * r) % N));
    uint32_t eps[2] = {0, 300};
    float mins[20], scale[20];
    oracle_sq8_train(x, N, d, mins, scale);
    uint8_t *codes = (uint8_t *)malloc((size_t)N * d);
    oracle_sq8_encode(x, N, d, mins, scale, codes);
    int64_t ids[9 * 6], stats[2];
    float dist[9 * 6];
    for (int metric = 0; metric < 2; ++metric)
        for (int sq = 0; sq < 2; ++sq) {
            oracle_diskann_search_batch(sq ? NULL : x, sq ? codes : NULL, mins, scale, N, d, adj, R, eps, 2, q, nq, k, L,
                                        metric, ids, dist, stats);
            CHECK(stats[0] > 0 && stats[1] > 0, "diskann stats");
            for (int i = 0; i < nq; ++i)
                for (int t = 0; t < k; ++t) {
                    CHECK(ids[i * k + t] >= 0 && ids[i * k + t] < N, "diskann id range");
                    if (t) CHECK(dist[i * k + t - 1] <= dist[i * k + t], "diskann order");
                }
        }
    free(x);
    free(q);
    free(adj);
    free(codes);
}

static void test_kmeans(void) {
    const int64_t n = 500;
    const int d = 12, nlist = 10;
    float *x = rand_mat(n, d);
    float cen[10 * 12];
    int64_t sizes[10];
    for (int metric = 0; metric < 2; ++metric)
        for (int init = 0; init < 2; ++init) {
            const int rc = oracle_kmeans_train(x, n, d, metric, nlist, 300, 5, 1234, init, cen, sizes);
            CHECK(rc == 0, "kmeans rc %d", rc);
            int64_t tot = 0;
            for (int l = 0; l < nlist; ++l) tot += sizes[l];
            CHECK(tot == 300 || tot == n, "kmeans sizes sum %lld", (long long)tot);
        }
    CHECK(oracle_kmeans_train(x, n, 0, 0, nlist, 0, 5, 1, 0, cen, sizes) < 0, "kmeans rejects d = 0");
    free(x);
}

int main(void) {
    test_flat();
    test_ivf();
    test_distances_and_sq8();
    test_diskann();
    test_kmeans();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("oracle self-test: all checks passed\n");
    return 0;
}
