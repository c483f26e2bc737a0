// hip_ann.cpp — C ABI (include/hip_ann.h) over the gfx950 Flat / IVFFlat search kernels.
//
// Reference behaviour mirrored here:
//   MetalIndexFlat::search (faiss-metal/src/MetalIndexFlat.mm:294-369): k <= 0 throws; empty
//     index / empty batch → (±inf, −1); effective_k = min(k, ntotal); labels int64.
//   MetalIndexFlat::add (MetalIndexFlat.mm:173-292): append rows, ‖x‖² computed on the device.
//   faiss_index.cpp:108-149 (EnsureGpuIndex) only needs create/search/free + availability.
#include "../../include/hip_ann.h"
#include "runtime.hpp"
#include "ivf.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>

using namespace hipann;

namespace {

void set_err(char *buf, int len, const char *msg) {
    if (!buf || len <= 0) return;
    std::strncpy(buf, msg, (size_t)len - 1);
    buf[len - 1] = '\0';
}

template <typename F>
int guard_int(char *eb, int el, F &&f) {
    try {
        return f();
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return -1;
}

template <typename F>
void *guard_ptr(char *eb, int el, F &&f) {
    try {
        return f();
    } catch (const std::exception &e) {
        set_err(eb, el, e.what());
    } catch (...) {
        set_err(eb, el, "hipann: unknown error");
    }
    return nullptr;
}

int g_device_count = -1;

int device_count() {
    if (g_device_count < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_device_count = n;
    }
    return g_device_count;
}

void require_device() { HIPANN_REQUIRE(device_count() > 0, "no HIP device"); }

std::vector<int> device_list(const int *devices, int ndev) {
    std::vector<int> v;
    if (!devices || ndev <= 0) v.push_back(0);
    else v.assign(devices, devices + ndev);
    for (int d : v) HIPANN_REQUIRE(d >= 0 && d < device_count(), "invalid device id " + std::to_string(d));
    return v;
}

}  // namespace

namespace hipann {
bool roctx_enabled() {
    static const bool on = [] { const char *e = std::getenv("HIPANN_ROCTX"); return e && std::atoi(e); }();
    return on;
}
void roctx_push(const char *name) { roctxRangePushA(name); }
void roctx_pop() { roctxRangePop(); }

std::vector<int> enable_peer_access(const std::vector<int> &devs) {
    std::vector<int> st(devs.size(), 2);
    if (devs.empty()) return st;
    const int d0 = devs[0];
    auto enable = [](int from, int to) -> bool {  // `from` may access `to`'s memory
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, from, to) != hipSuccess || !can) return false;
        DeviceGuard g(from);
        const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) {
            (void)hipGetLastError();  // clear the sticky-free "already enabled" status
            return true;
        }
        return e == hipSuccess;
    };
    for (size_t p = 1; p < devs.size(); ++p) {
        if (devs[p] == d0) continue;
        st[p] = enable(d0, devs[p]) && enable(devs[p], d0) ? 1 : 0;
    }
    return st;
}
}  // namespace hipann

namespace {

hipStream_t make_stream(int dev) {
    DeviceGuard g(dev);
    hipStream_t s;
    HIPANN_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

constexpr int kFusedMaxK = 64;   // fused GEMM / scan lists: one element per lane
constexpr int kBlasThreshold = 20;  // FAISS distance_compute_blas_threshold
constexpr int64_t kSmallTable = 16384;  // rows: below this, GEMM keys + per-query selection

// Grow `b` to at least `need` bytes keeping its first `keep` bytes (device-to-device on `st`).
void grow_keep(DevBuf &b, size_t need, size_t keep, int dev, hipStream_t st) {
    if (b.p && need <= b.bytes) return;
    DevBuf nb;
    nb.ensure(need, dev);
    if (b.p && keep) HIPANN_CHECK(hipMemcpyAsync(nb.p, b.p, std::min(keep, b.bytes), hipMemcpyDeviceToDevice, st));
    HIPANN_CHECK(hipStreamSynchronize(st));  // the old buffer is freed on return
    std::swap(b.p, nb.p);
    std::swap(b.bytes, nb.bytes);
    std::swap(b.device, nb.device);
}

float bits_to_float(unsigned u) {
    float v;
    std::memcpy(&v, &u, sizeof(v));
    return v;
}

// Append rows to a shard's owned storage (capacity doubling, as MetalIndexFlat::add does, MetalIndexFlat.mm:255-269).
// The search images built from the rows (int8 / bf16 tiles, per-row int8 scales) grow with the same capacity and
// only the tiles holding new rows are re-tiled; the exact forms' bound terms (max ‖x‖², the largest int8 / bf16 row
// residual) become running maxima over the new rows — an append costs the appended rows, not the table.
void shard_append(FlatShard &sh, int d, int metric, const float *x_host, const float *x_dev, int64_t n) {
    if (n <= 0) return;
    DeviceGuard g(sh.device);
    FenceScope fs(sh.fence, sh.stream, sh.device);  // searches still running on other streams read sh.xb
    hipStream_t st = sh.stream;
    const int64_t n0 = sh.n, need = sh.n + n;
    if (need > sh.cap || !sh.owns) {
        const int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1024, sh.cap * 2));
        DevBuf nb;
        nb.ensure((size_t)cap * d * sizeof(float), sh.device);
        if (sh.n > 0)
            HIPANN_CHECK(hipMemcpyAsync(nb.get<float>(), sh.xb, (size_t)sh.n * d * sizeof(float), hipMemcpyDeviceToDevice,
                                        st));
        HIPANN_CHECK(hipStreamSynchronize(st));
        std::swap(sh.xb_buf.p, nb.p);
        std::swap(sh.xb_buf.bytes, nb.bytes);
        sh.xb_buf.device = sh.device;
        sh.xb = sh.xb_buf.get<float>();
        sh.cap = cap;
        sh.owns = true;
        if (metric == kL2) grow_keep(sh.xn, (size_t)cap * sizeof(float), (size_t)sh.n * sizeof(float), sh.device, st);
    }
    float *dst = sh.xb + n0 * (int64_t)d;
    if (x_host)
        HIPANN_CHECK(hipMemcpyAsync(dst, x_host, (size_t)n * d * sizeof(float), hipMemcpyHostToDevice, st));
    else
        HIPANN_CHECK(hipMemcpyAsync(dst, x_dev, (size_t)n * d * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (metric == kL2) launch_row_norms(dst, n, d, sh.xn.get<float>() + n0, st);
    sh.n = need;
    // the images and bound terms, when built: tiles from the first one holding a new row to the end
    const bool upd = sh.xmax2 >= 0.f || sh.xi8_ok || sh.xb16_ok;
    if (upd) {
        const int R = flat_bf16_tile_rows();
        const int64_t t0 = n0 / R;                  // first tile with a new row (tiles before it are unchanged)
        const int64_t capr = ceil_div(sh.cap, (int64_t)R) * R;
        sh.app_stat.ensure(sizeof(unsigned) * 4, sh.device);
        unsigned *stat = sh.app_stat.get<unsigned>();
        HIPANN_CHECK(hipMemsetAsync(stat, 0, sizeof(unsigned) * 4, st));
        sh.tmpnorm.ensure(sizeof(float) * (size_t)n, sh.device);
        if (sh.xmax2 >= 0.f) {
            const float *xn_new = sh.xn.get<float>() + n0;
            if (metric != kL2) {
                launch_row_norms(dst, n, d, sh.tmpnorm.get<float>(), st);
                xn_new = sh.tmpnorm.get<float>();
            }
            launch_ivf_max_norm(xn_new, n, stat + 0, st);
        }
        if (sh.xi8_ok) {
            const size_t tb = flat_i8_img_bytes(R, d, R);  // one tile
            grow_keep(sh.xi8, flat_i8_img_bytes(capr, d, R), (size_t)t0 * tb, sh.device, st);
            grow_keep(sh.xscale, sizeof(float) * (size_t)capr, sizeof(float) * (size_t)n0, sh.device, st);
            float *rs = sh.tmpnorm.get<float>();
            launch_i8_row_scale(dst, n, d, sh.xscale.get<float>() + n0, rs, st);
            launch_ivf_max_norm(rs, n, stat + 1, st);
            launch_i8_tile_rows(sh.xb + t0 * R * (int64_t)d, sh.xscale.get<float>() + t0 * R, sh.n - t0 * R, d, R,
                                static_cast<char *>(sh.xi8.p) + (size_t)t0 * tb, st);
        }
        if (sh.xb16_ok) {
            const size_t tb = flat_bf16_img_bytes(R, d, R);
            grow_keep(sh.xb16, flat_bf16_img_bytes(capr, d, R), (size_t)t0 * tb, sh.device, st);
            float *rs = sh.tmpnorm.get<float>();
            launch_b16_row_residual2(dst, n, d, rs, st);
            launch_ivf_max_norm(rs, n, stat + 2, st);
            launch_b16_tile_rows(sh.xb + t0 * R * (int64_t)d, sh.n - t0 * R, d, R,
                                 static_cast<char *>(sh.xb16.p) + (size_t)t0 * tb, st);
        }
        unsigned hs[4] = {0u, 0u, 0u, 0u};
        HIPANN_CHECK(hipMemcpyAsync(hs, stat, sizeof(hs), hipMemcpyDeviceToHost, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
        if (sh.xmax2 >= 0.f) sh.xmax2 = std::max(sh.xmax2, bits_to_float(hs[0]));
        if (sh.xi8_ok) sh.i8_rxmax = std::max(sh.i8_rxmax, bits_to_float(hs[1]));
        if (sh.xb16_ok) sh.bf16_rxmax = std::max(sh.bf16_rxmax, std::sqrt(bits_to_float(hs[2])) * 1.0001f);
    } else {
        HIPANN_CHECK(hipStreamSynchronize(st));
    }
}

}  // namespace

namespace hipann {

FlatIndex::~FlatIndex() {
    for (auto &s : shards) {
        DeviceGuard g(s->device);
        if (s->done) (void)hipEventDestroy(s->done);
        if (s->stream) (void)hipStreamDestroy(s->stream);
    }
}

// k > 64: distance keys for a column chunk into HBM (GEMM or direct scan, same forms as the fused
// path), per-(row, segment) S-slot wave lists, and a running merge across chunks.
static void flat_shard_search_bigk(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, const float *qn, int k,
                                   int kout, float *D, int64_t *I, hipStream_t st) {
    const int d = ix.d, metric = ix.metric;
    const float out_sign = metric == kIP ? -1.f : 1.f;
    const int64_t budget = (int64_t)256 << 20;  // bytes of keys per chunk
    int64_t C = std::max<int64_t>(1024, budget / (4 * std::max<int64_t>(nq, 1)));
    C = std::min<int64_t>(C, sh.n);
    C = (C + 127) / 128 * 128;
    const int64_t seg_len = 8192;
    const int nseg = (int)ceil_div(C, seg_len);
    sh.keys.ensure((size_t)nq * C * sizeof(float), sh.device);
    sh.part_d.ensure((size_t)(nseg + 1) * nq * k * sizeof(float), sh.device);
    sh.part_i.ensure((size_t)(nseg + 1) * nq * k * sizeof(int), sh.device);
    if (sh.n <= C) {  // one chunk (an IVF coarse quantizer): the segment lists go straight to the output merge
        {
            ScopedTiming t(ix.timer_main, st);
            if (nq < kBlasThreshold)
                launch_flat_scan_keys(xq, (int)nq, sh.xb, sh.n, d, metric, sh.keys.get<float>(), C, st);
            else
                launch_flat_gemm_keys(xq, qn, nq, sh.xb, sh.xn.get<float>(), sh.n, d, metric, sh.keys.get<float>(), C,
                                      st, sh.keys_bf3);
        }
        {  // kout ≤ 256: one wave selects the whole row and writes the output (no segment lists, no merge)
            ScopedTiming t(ix.timer_merge, st);
            // (short rows only: a long row would be one wave's serial inserts — the segment path spreads it)
            if (sh.n <= kSmallTable && launch_rows_select_out(sh.keys.get<float>(), C, sh.n, nq, k, kout,
                                                              sh.label_offset, out_sign, D, I, st, sh.plan_hook))
                return;
        }
        // short rows: 256-column segments, so a 1024-centroid row is selected by 4 waves, not 1
        const int64_t sl = sh.n <= seg_len && k <= 64 ? 256 : seg_len;
        const int ns = (int)ceil_div(sh.n, sl);
        sh.part_d.ensure((size_t)ns * nq * k * sizeof(float), sh.device);
        sh.part_i.ensure((size_t)ns * nq * k * sizeof(int), sh.device);
        launch_rows_topk(sh.keys.get<float>(), C, sh.n, nq, sl, ns, k, 0, sh.part_d.get<float>(), sh.part_i.get<int>(),
                         st);
        ScopedTiming t(ix.timer_merge, st);
        launch_merge_parts<int>(sh.part_d.get<float>(), sh.part_i.get<int>(), ns, nq, k, kout, sh.label_offset, 1.f,
                                out_sign, D, I, st);
        return;
    }
    sh.run_d.ensure((size_t)nq * k * sizeof(float), sh.device);
    sh.run_i.ensure((size_t)nq * k * sizeof(int), sh.device);
    // running best starts empty: part 0 = pads
    HIPANN_CHECK(hipMemsetAsync(sh.part_i.p, 0xff, (size_t)nq * k * sizeof(int), st));
    for (int64_t c0 = 0; c0 < sh.n; c0 += C) {
        const int64_t cn = std::min<int64_t>(C, sh.n - c0);
        {
            ScopedTiming t(ix.timer_main, st);
            if (nq < kBlasThreshold)
                launch_flat_scan_keys(xq, (int)nq, sh.xb + c0 * d, cn, d, metric, sh.keys.get<float>(), C, st);
            else
                launch_flat_gemm_keys(xq, qn, nq, sh.xb + c0 * d, sh.xn.get<float>() + c0, cn, d, metric,
                                      sh.keys.get<float>(), C, st);
        }
        const int ns = (int)ceil_div(cn, seg_len);
        launch_rows_topk(sh.keys.get<float>(), C, cn, nq, seg_len, ns, k, (int)c0,
                         sh.part_d.get<float>() + (size_t)nq * k, sh.part_i.get<int>() + (size_t)nq * k, st);
        // merge [running best, ns segment partials] → running best (then back into part 0)
        launch_merge_raw(sh.part_d.get<float>(), sh.part_i.get<int>(), ns + 1, nq, k, sh.run_d.get<float>(),
                         sh.run_i.get<int>(), st);
        HIPANN_CHECK(hipMemcpyAsync(sh.part_d.p, sh.run_d.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToDevice, st));
        HIPANN_CHECK(hipMemcpyAsync(sh.part_i.p, sh.run_i.p, (size_t)nq * k * sizeof(int), hipMemcpyDeviceToDevice, st));
    }
    ScopedTiming t(ix.timer_merge, st);
    launch_merge_parts<int>(sh.run_d.get<float>(), sh.run_i.get<int>(), 1, nq, k, kout, sh.label_offset, 1.f, out_sign,
                            D, I, st);
}

// The shard's tiled int8 image (form kFlatI8Exact): per-row scales max|x|/127, the rows' int8 units in the bf16
// image's tile geometry, and the largest row residual ‖x − s·x̂‖ (the rerank bound's row term).  Built once.
static void ensure_i8_image(FlatIndex &ix, FlatShard &sh, int d, hipStream_t st) {
    if (sh.xi8_ok) return;
    sh.xi8.ensure(flat_i8_img_bytes(sh.n, d, flat_bf16_tile_rows()), sh.device);
    sh.xscale.ensure(sizeof(float) * (size_t)sh.n, sh.device);
    sh.tmpnorm.ensure(sizeof(float) * (size_t)sh.n, sh.device);
    launch_i8_row_scale(sh.xb, sh.n, d, sh.xscale.get<float>(), sh.tmpnorm.get<float>(), st);
    launch_i8_tile_rows(sh.xb, sh.xscale.get<float>(), sh.n, d, flat_bf16_tile_rows(), sh.xi8.p, st);
    sh.nflag.ensure(sizeof(int), sh.device);
    launch_ivf_max_norm(sh.tmpnorm.get<float>(), sh.n, sh.nflag.get<unsigned>(), st);  // max of non-negative
    unsigned bits = 0;
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    ++ix.host_syncs;
    sh.tmpnorm.release();
    std::memcpy(&sh.i8_rxmax, &bits, sizeof(float));
    sh.xi8_ok = true;
}

// Search one shard: queries already on the shard's device.  Writes D (nq×kout fp32: raw distances,
// ±inf pads) and I (nq×kout int64 labels, −1 pads) on the same device, asynchronously on `st`.
// max‖x‖² of the shard (once per row set): the exact form's error bound
static float flat_xmax2(FlatIndex &ix, FlatShard &sh, int d, hipStream_t st) {
    if (sh.xmax2 >= 0.f) return sh.xmax2;
    const float *xn = sh.xn.get<float>();
    if (!xn) {
        sh.tmpnorm.ensure(sizeof(float) * (size_t)std::max<int64_t>(sh.n, 1), sh.device);
        launch_row_norms(sh.xb, sh.n, d, sh.tmpnorm.get<float>(), st);
        xn = sh.tmpnorm.get<float>();
    }
    sh.nflag.ensure(sizeof(int), sh.device);
    launch_ivf_max_norm(xn, sh.n, sh.nflag.get<unsigned>(), st);
    unsigned bits = 0;
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    ++ix.host_syncs;
    sh.tmpnorm.release();
    float v;
    std::memcpy(&v, &bits, sizeof(v));
    sh.xmax2 = v;
    return v;
}

// The bounded passes' plan: tile boundaries 0 = b₀ < b₁ < … < b_P = tps within every split.  Pass 0 admits the
// rows under the seed (the k-th of S sample keys): ≈ k·(b₁·nsplit·rows)/S candidates per query; pass p ≥ 1 runs
// under the k-th over every earlier row: ≈ k·(b_{p+1} − b_p)/b_p.  Every candidate costs a scattered store and
// the epilogue's slow path (measured ≈ 0.54 µs per candidate per query per 1024-query batch: C2 and 10M pass-A
// sweeps, profiles/r04/passa_sweep_r04.txt), every pass ≈ 55 µs (its pipeline fill + the bound kernel), so P and
// geometric boundaries b_p ≈ (S/(nsplit·rows))·g^p, g = (N/S)^{1/P}, minimise candidates·nq·0.54 ns + P·55 µs.
// HIPANN_FLAT_PASSES pins P (A/B).
static std::vector<int64_t> flat_pass_plan(int64_t tps, int64_t nsplit, int64_t tile_rows, int64_t sample, int k,
                                           int64_t nq) {
    static const int forced = [] { const char *e = std::getenv("HIPANN_FLAT_PASSES"); return e ? std::atoi(e) : 0; }();
    const double unit = (double)sample / ((double)nsplit * (double)tile_rows);  // the sample in tiles per split
    std::vector<int64_t> best{0, tps};
    double best_cost = 1e300;
    for (int P = 1; P <= 6; ++P) {
        if (forced > 0 && P != forced) continue;
        std::vector<int64_t> b{0};
        const double g = std::pow((double)tps / unit, 1.0 / P);
        for (int p = 1; p < P; ++p) {
            const int64_t t = std::llround(unit * std::pow(g, p));
            if (t > b.back() && t < tps) b.push_back(t);
        }
        b.push_back(tps);
        if ((int)b.size() != P + 1) continue;  // too few tiles for P passes
        double cand = k * (double)b[1] / unit;
        for (size_t p = 1; p + 1 < b.size(); ++p) cand += k * (double)(b[p + 1] - b[p]) / (double)b[p];
        const double cost = cand * (double)nq * 0.54e-9 + P * 55e-6;
        if (cost < best_cost) { best_cost = cost; best = b; }
    }
    return best;
}

// The flag count of the launch phase's bound check into the shard's pinned host word (a copy kernel through its
// device mapping, no DMA round trip), then a fresh token into the word after it; the host reads the count after
// its next synchronisation with `st` (or once the token arrives, wait_posted).
static void flag_readback(FlatShard &sh, hipStream_t st) {
    if (sh.h_nflag.ensure(2 * sizeof(unsigned), hipHostMallocCoherent)) sh.h_nflag.get<unsigned>()[1] = sh.flag_seq;
    launch_post_words(sh.nflag.p, sh.h_nflag.p, 1, ++sh.flag_seq, st);
}

// Launch phase of a shard search: every kernel of the search up to the exact forms' flag count, enqueued on `st`
// without a host synchronisation.  pend says what flat_shard_finish has left to do (kNone: the output is complete
// once `st` drains).
static void flat_shard_launch(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                              int64_t *I, hipStream_t st, int form_override, FlatPending &pend) {
    pend = FlatPending{};
    DeviceGuard g(sh.device);
    const int d = ix.d, metric = ix.metric;
    const float out_sign = metric == kIP ? -1.f : 1.f;
    HIPANN_REQUIRE(k <= HIPANN_MAX_K, "k larger than HIPANN_MAX_K");
    // set below when this call computes ‖q‖² into sh.qn (or already: the caller prepared it, qn_given)
    sh.qn_of = sh.qn_given == xq && sh.qn_given_nq == nq ? xq : nullptr;
    sh.qn_nq = nq;
    if (nq <= 0) return;
    if (sh.n == 0) {  // no rows: pads only
        launch_merge_parts<int>(nullptr, nullptr, 0, nq, k, kout, sh.label_offset, 1.f, out_sign, D, I, st);
        return;
    }
    HIPANN_REQUIRE(sh.n <= (int64_t)0x7ffffffe, "shard larger than 2^31-2 rows");
    // Large k, or a small table (an IVF coarse quantizer: nq x nlist keys are a few MB): the GEMM writes
    // the key matrix and one wave per query selects — the fused epilogue would spend its time
    // filling empty lists, one query tile per CU.
    // nq < 20 on a table of ≤ 1024 rows (the coarse quantizer of the extension's nq = 1 call): direct-form
    // keys over ≥ 16-row waves + one bitwise select per query row (the fused scan's nparts × k partial
    // lists took one wave 47 µs to merge at nlist 1024)
    if (k > kFusedMaxK || (nq >= kBlasThreshold && sh.n <= kSmallTable) ||
        (nq < kBlasThreshold && sh.n <= 1024 && kout <= 64 && scan_smem_bytes((int)nq, d) <= 64 * 1024)) {
        const float *qn = nullptr;
        if (nq >= kBlasThreshold && metric == kL2) {
            if (!(sh.qn_given == xq && sh.qn_given_nq == nq)) {
                sh.qn.ensure((size_t)nq * sizeof(float), sh.device);
                launch_row_norms(xq, nq, d, sh.qn.get<float>(), st);
            }
            qn = sh.qn.get<float>();
            sh.qn_of = xq;
            sh.qn_nq = nq;
        }
        flat_shard_search_bigk(ix, sh, nq, xq, qn, k, kout, D, I, st);
        return;
    }
    // nq < 20 on a large table (the extension's per-query calls, faiss_index.cpp:737): form 5's int8 image as the
    // filter — flat_i8_scan (a quarter of the fp32 rows' bytes), 64 candidates per query, the exact direct-form
    // rerank with the int8 residual bound; queries it cannot certify re-run on the fp32 direct scan below.
    // HIPANN_FLAT_I8_SMALL=0 keeps every nq < 20 call on the fp32 scan (A/B).
    static const bool i8_small_env = [] { const char *e = std::getenv("HIPANN_FLAT_I8_SMALL"); return !e || std::atoi(e); }();
    const int req_form = form_override >= 0 ? form_override : ix.form;
    if (nq <= flat_i8_scan_max_nq() && req_form == kFlatI8Exact && i8_small_env && sh.n >= 65536 && d <= 1024 &&
        kout <= flat_i8_scan_k() && k <= flat_i8_scan_k()) {
        const int kf = flat_i8_scan_k();
        ensure_i8_image(ix, sh, d, st);
        const float xmax2 = flat_xmax2(ix, sh, d, st);
        const int64_t nw = flat_i8_scan_waves(sh.n);
        const int G = (int)std::min<int64_t>(64, nw);
        const float *qn = nullptr;
        if (metric == kL2) {
            sh.qn.ensure((size_t)nq * sizeof(float), sh.device);
            launch_row_norms(xq, nq, d, sh.qn.get<float>(), st);
            qn = sh.qn.get<float>();
        }
        sh.qscale.ensure(sizeof(float) * (size_t)nq, sh.device);
        sh.qres.ensure(sizeof(float) * (size_t)nq, sh.device);
        sh.qimg.ensure((size_t)nq * flat_i8_nk(d) * 4 * 16, sh.device);
        sh.part_d.ensure((size_t)nw * nq * kf * sizeof(float), sh.device);
        sh.part_i.ensure((size_t)nw * nq * kf * sizeof(int), sh.device);
        sh.mid_d.ensure((size_t)G * nq * kf * sizeof(float), sh.device);
        sh.mid_i.ensure((size_t)G * nq * kf * sizeof(long long), sh.device);
        {
            ScopedTiming t(ix.timer_main, st);
            launch_flat_i8_scan(xq, nq, d, metric, sh.xi8.p, sh.xscale.get<float>(), sh.xn.get<float>(), sh.n,
                                sh.qscale.get<float>(), sh.qres.get<float>(), qn, sh.qimg.p, sh.part_d.get<float>(),
                                sh.part_i.get<int>(), nw, st);
        }
        sh.nflag.ensure(sizeof(int), sh.device);
        sh.flagged.ensure(sizeof(int) * (size_t)nq, sh.device);
        HIPANN_CHECK(hipMemsetAsync(sh.nflag.p, 0, sizeof(int), st));
        {
            ScopedTiming t(ix.timer_merge, st);
            float *md = sh.mid_d.get<float>();
            int *mi = reinterpret_cast<int *>(sh.mid_i.p);
            launch_flat_i8_group_merge(sh.part_d.get<float>(), sh.part_i.get<int>(), (int)nw, (int)nq, G, md, mi, st);
            launch_ivf_rerank(md, mi, nullptr, G, nq, kf, kout, metric, xq, sh.xb, d, nullptr, sh.n, sh.label_offset,
                              xmax2, D, I, sh.nflag.get<int>(), sh.flagged.get<int>(), st, kSplit2Eps, sh.i8_rxmax,
                              sh.qres.get<float>());
        }
        if (form_override < 0) {
            ix.last_form = kFlatI8Exact;
            ix.last_kfilt = kf;
            ix.last_sublists = 0;
        }
        // the flagged count goes to the host with the results; the uncertified queries re-run on the fp32 direct
        // scan in flat_shard_finish
        pend = FlatPending{};
        pend.kind = FlatPending::kSmallI8;
        pend.nq = nq;
        pend.xq = xq;
        pend.k = k;
        pend.kout = kout;
        pend.D = D;
        pend.I = I;
        flag_readback(sh, st);
        return;
    }
    if (nq < kBlasThreshold) {
        if (form_override < 0) {
            ix.last_form = kFlatFp32;  // the direct form
            ix.last_kfilt = 0;
            ix.last_sublists = 0;
        }
        // direct form (fvec_L2sqr / fvec_inner_product)
        // ≥ 512 rows per wave on large tables; small ones (the IVF coarse quantizer's 1024 centroids at
        // nq = 1) are spread over waves of ≥ 16 rows (2 waves of 512 rows took 234 us for 1024 × 768)
        int64_t nwaves = std::min<int64_t>(8192, std::max<int64_t>(std::min<int64_t>(256, ceil_div(sh.n, 16)),
                                                                   ceil_div(sh.n, 512)));
        const int64_t rpw = ceil_div(sh.n, nwaves);
        nwaves = ceil_div(sh.n, rpw);
        const int64_t nw_alloc = ceil_div(nwaves, 4) * 4;
        // the scan holds its queries in ≤ 64 KiB of LDS: larger d·nq runs as several query chunks (d = 1536 fits 10
        // queries; one query up to d = 16384)
        int qc = (int)nq;
        while (qc > 1 && scan_smem_bytes(qc, d) > 64 * 1024) --qc;
        HIPANN_REQUIRE(scan_smem_bytes(qc, d) <= 64 * 1024, "dimension too large for the scan path");
        sh.part_d.ensure((size_t)nw_alloc * qc * k * sizeof(float), sh.device);
        sh.part_i.ensure((size_t)nw_alloc * qc * k * sizeof(int), sh.device);
        const int groups = (int)std::min<int64_t>(256, ceil_div(nw_alloc, 32));
        if (nw_alloc > 256) {
            sh.mid_d.ensure(sizeof(float) * (size_t)groups * qc * kout, sh.device);
            sh.mid_i.ensure(sizeof(long long) * (size_t)groups * qc * kout, sh.device);
        }
        for (int64_t q0 = 0; q0 < nq; q0 += qc) {
            const int64_t nc = std::min<int64_t>(qc, nq - q0);
            {
                ScopedTiming t(ix.timer_main, st);
                launch_flat_scan_topk(xq + q0 * d, (int)nc, sh.xb, sh.n, d, metric, k, (int)nw_alloc, rpw,
                                      sh.part_d.get<float>(), sh.part_i.get<int>(), st);
            }
            ScopedTiming t(ix.timer_merge, st);
            if (nw_alloc > 256) {
                // thousands of per-wave lists: groups of ~32 merged by one wave each, then the group lists by one
                // 4-wave block per query (one wave per query took ~1 ms for 8192 lists at 10M rows, nq = 1)
                launch_merge_parts_2level<int>(sh.part_d.get<float>(), sh.part_i.get<int>(), (int)nw_alloc, nc, k, kout,
                                               sh.label_offset, 1.f, out_sign, D + q0 * kout, I + q0 * kout,
                                               sh.mid_d.get<float>(), sh.mid_i.get<long long>(), groups, st);
            } else {
                launch_merge_parts<int>(sh.part_d.get<float>(), sh.part_i.get<int>(), (int)nw_alloc, nc, k, kout,
                                        sh.label_offset, 1.f, out_sign, D + q0 * kout, I + q0 * kout, st);
            }
        }
        return;
    }
    // BLAS form: ‖q‖² + ‖x‖² − 2 q·x on fp32 MFMA.  ‖q‖² is launched by qn_now() ahead of its first reader (the int8
    // bounded passes compute it inside their query preparation instead, the same bits)
    const float *qn = nullptr;
    bool qn_launch = false;
    if (metric == kL2) {
        if (!(sh.qn_given == xq && sh.qn_given_nq == nq)) {
            sh.qn.ensure((size_t)nq * sizeof(float), sh.device);
            qn_launch = true;
        }
        qn = sh.qn.get<float>();
        sh.qn_of = xq;
        sh.qn_nq = nq;
    }
    auto qn_now = [&]() {
        if (qn_launch) launch_row_norms(xq, nq, d, sh.qn.get<float>(), st);
        qn_launch = false;
    };
    int form = form_override >= 0 ? form_override : ix.form;
    static const bool seed_env = [] { const char *e = std::getenv("HIPANN_FLAT_BF16_SEED"); return !e || std::atoi(e); }();
    // The exact forms keep kf candidates per query (per split and query on the list kernels) as the filter; the
    // rerank returns kout.  kout ≤ kRerankMaxK: kf = 32 (the bf16 image: at 10M × 768 the 10th and 16th distances
    // are ≈2 apart, inside its rounding bound ≈1.3, the 10th and 32nd ≈5; the split scan: IP 32, L2 16).  Larger
    // kout (request_k = k + |tombstones|, faiss_index.cpp:713-715): kf = min(64, max(base, 2·kout)).  The list
    // kernels hold kf in LDS (capped by their launchers' LDS budget) and need kf ≥ kout + 4 of margin; the bounded
    // passes take any kout ≤ kf ≤ 64 — a query whose kout-th distance is within the bound of the kf-th key goes to
    // the all-candidate rerank, certified against the pass bound.  Otherwise: the 3-term split (fp32-level).
    int kf = 0;
    bool bounded = false;
    // kFlatI8Exact runs only as the bounded passes (256-query blocks, >= 512K rows, d <= 1024 so the int32 sums
    // convert to fp32 exactly); elsewhere the bf16 image's paths
    if (form == kFlatI8Exact &&
        !(flat_bf16_resumable(nq, d, 64) && seed_env && sh.n >= 8 * 65536 && d <= 1024))
        form = kFlatBf16Exact;
    if (form == kFlatI8Exact) {
        // the int8 rounding bound is ≈3× the bf16 one (E ≈ 4.4 against 1.3-1.7 at 768 dims on U(-1, 1)): a
        // 64-deep filter keeps the 10th distance clear of it (the 10th-to-32nd gap is ≈5, the 10th-to-64th ≈8)
        kf = 64;
        bounded = true;
    } else if (form == kFlatSplit2Exact || form == kFlatBf16Exact) {
        const int base = metric == kIP || form == kFlatBf16Exact ? kFlatRerankKIP : kRerankK;
        kf = kout <= kRerankMaxK ? base : std::min(64, std::max(base, 2 * kout));
        if (form == kFlatBf16Exact) {
            bounded = flat_bf16_resumable(nq, d, kf) && seed_env && sh.n >= 8 * 65536;
            if (!bounded) kf = std::min(kf, flat_bf16_topk_kmax(nq));
        } else {
            kf = std::min(kf, flat_gemm_topk_bf_kmax(2));
        }
    }
    const bool exact = kf > 0 && (kout <= kRerankMaxK || (bounded ? kout <= kf : kout + 4 <= kf));
    if (kf > 0 && !exact) form = kFlatSplit3;
    const int k_user = k;
    if (exact) k = kf;
    // the split scans' LDS lists hold fewer rows at 3 terms (k <= 38 at 8 waves): a longer list takes the fp32
    // matrix cores (exact fp32 products, lists up to 64)
    if ((form == kFlatSplit3 || form == kFlatSplit2) && k > flat_gemm_topk_bf_kmax(form == kFlatSplit3 ? 3 : 2))
        form = kFlatFp32;
    if (form_override < 0) {
        ix.last_form = form;
        ix.last_kfilt = exact ? kf : 0;
        ix.last_sublists = 0;
    }
    int64_t nsplit;
    bool flags_ready = false;  // the bounded passes' select already reset nflag and flagged overflows
    // the bounded passes' candidate buffers and bound, for the flagged queries' second rerank
    const float *cr_d = nullptr, *cr_bound = nullptr;
    const int *cr_i = nullptr, *cr_n = nullptr;
    int cr_nsplit = 0, cr_cap = 0;
    // the exact forms' max ‖x‖² (cached; its first computation uses sh.nflag as scratch, so before any flags)
    const float xmax2 = exact ? flat_xmax2(ix, sh, d, st) : 0.f;
    const bool i8 = form == kFlatI8Exact;
    float rxmax = sh.bf16_rxmax;  // the rerank bound's row term of the form that filtered
    if (i8) {
        // one int8 product per element (int32 sums) over a tiled int8 image with per-row scales, built once
        ensure_i8_image(ix, sh, d, st);
        rxmax = sh.i8_rxmax;
    }
    // HIPANN_I8_PREP_FUSED=0 (A/B): the int8 query preparation as row_norms + i8_row_scale + i8_tile_rows
    static const bool prep_fused = [] { const char *e = std::getenv("HIPANN_I8_PREP_FUSED"); return !e || std::atoi(e); }();
    const bool i8_prep = i8 && bounded && seed_env && sh.n >= 8 * 65536 && prep_fused;
    if (!i8_prep) qn_now();
    if (form == kFlatBf16Exact || i8) {
        // one plain bf16 product per element over the tiled bf16 image (flat_bf16.hip), built once
        if (!i8 && !sh.xb16_ok) {
            sh.xb16.ensure(flat_bf16_img_bytes(sh.n, d, flat_bf16_tile_rows()), sh.device);
            launch_b16_tile_rows(sh.xb, sh.n, d, flat_bf16_tile_rows(), sh.xb16.p, st);
            // the rows' largest bf16 rounding residual ‖x̂ − x‖ (the rerank's bound)
            sh.tmpnorm.ensure(sizeof(float) * (size_t)sh.n, sh.device);
            launch_b16_row_residual2(sh.xb, sh.n, d, sh.tmpnorm.get<float>(), st);
            sh.nflag.ensure(sizeof(int), sh.device);
            launch_ivf_max_norm(sh.tmpnorm.get<float>(), sh.n, sh.nflag.get<unsigned>(), st);
            unsigned bits = 0;
            HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
            HIPANN_CHECK(hipStreamSynchronize(st));  // later searches may run on other streams
            ++ix.host_syncs;
            sh.tmpnorm.release();
            float r2;
            std::memcpy(&r2, &bits, sizeof(r2));
            sh.bf16_rxmax = std::sqrt(r2) * 1.0001f;
            sh.xb16_ok = true;
        }
        const int W = flat_bf16_waves(nq);
        const int64_t nqt = ceil_div(nq, 32 * W);
        // the scan's operand images, chunk count and (int8) scales
        const void *ximg = i8 ? sh.xi8.p : sh.xb16.p;
        const int nk = i8 ? flat_i8_nk(d) : (int)ceil_div(d, 32);
        const float *qsc = nullptr, *xsc = i8 ? sh.xscale.get<float>() : nullptr;
        const int64_t ntiles = ceil_div(sh.n, flat_bf16_tile_rows());
        static const int64_t blocks_env = [] {
            const char *e = std::getenv("HIPANN_FLAT_BF16_BLOCKS");  // A/B: target grid size
            return e ? (int64_t)std::atoll(e) : (int64_t)0;
        }();
        // one round of resident blocks (W = 8 / 4: one block per CU; W = 2: two) — fewer, longer splits admit
        // fewer candidates into the per-split lists (≈ k·ln(rows / k) per list), the epilogue's slow path
        nsplit = std::max<int64_t>(1, ceil_div(blocks_env > 0 ? blocks_env : (W == 2 ? 512 : 256), nqt));
        nsplit = std::min<int64_t>(nsplit, ntiles);
        const int64_t tps = ceil_div(ntiles, nsplit);
        nsplit = ceil_div(ntiles, tps);
        HIPANN_REQUIRE(nqt * nsplit < (int64_t)0x7fffffff, "grid too large");
        sh.part_d.ensure((size_t)nsplit * nq * k * sizeof(float), sh.device);
        sh.part_i.ensure((size_t)nsplit * nq * k * sizeof(int), sh.device);
        sh.qimg.ensure(i8 ? flat_i8_img_bytes(nq, d, 32 * W) : flat_bf16_img_bytes(nq, d, 32 * W), sh.device);
        // seed bound (large tables): the k-th best key of each query over a sample of the first rows.  Bounded
        // passes (below): the sample's keys from the same kernel in its keys mode (a dense nq × S matrix, one
        // tile per block) and their k-th order statistic (flat_keys_kth); otherwise the 32-dim list kernel over
        // 64K rows and flat_bf16_seed (its lists start empty: every row an insert, ≈1 ms at 1024 queries — what
        // the keys mode replaces).  The main passes then admit only keys ≤ that bound.
        const bool seeded = seed_env && sh.n >= 8 * 65536;
        static const int64_t pass_div = [] {
            const char *e = std::getenv("HIPANN_FLAT_PASS_A");  // A/B: two passes, 1/x of each split in pass A
            return e ? (int64_t)std::atoll(e) : (int64_t)-1;
        }();
        static const int64_t sample_env = [] {
            const char *e = std::getenv("HIPANN_FLAT_SAMPLE");  // A/B: rows of the seed sample (multiple of 256)
            return e ? (int64_t)std::atoll(e) : (int64_t)16384;
        }();
        const int64_t sample = std::max<int64_t>(256, std::min<int64_t>(sample_env / 256 * 256, flat_keys_kth_max()));
        // the passes' tile boundaries within every split: pass p scans tiles [pb[p], pb[p+1]) under the bound
        // from everything before it (the seed for pass 0)
        const std::vector<int64_t> pb = pass_div >= 0
            ? std::vector<int64_t>(pass_div > 1 && tps / pass_div >= 1 ? std::vector<int64_t>{0, tps / pass_div, tps}
                                                                     : std::vector<int64_t>{0, tps})
            : flat_pass_plan(tps, nsplit, flat_bf16_tile_rows(), sample, k, nq);
        // per-(query, split) candidate capacity from the expected fill: pass 0 admits ≈ k·rows₀/S per cell (keys ≤
        // the k-th of S sample rows), pass p ≈ k·rows_p/(nsplit·rows_<p) (the k-th over all earlier rows); 3× + 32
        // of headroom (clustered 12.5M IP rows peaked at 2.3× the mean), a multiple of 32.
        double fill = k * (double)(pb[1] * flat_bf16_tile_rows()) / (double)sample;
        for (size_t p = 1; p + 1 < pb.size(); ++p)
            fill += k * (double)(pb[p + 1] - pb[p]) / ((double)pb[p] * (double)nsplit);
        const int cap = (int)std::min<double>(1 << 20, (double)ceil_div((int64_t)(3.0 * fill + 32.0), 32) * 32);
        const size_t ncell = (size_t)nq * nsplit;
        // the keys-mode seed pass runs per chunk of 1024 queries (4 query tiles) through one 64 MB slab of keys
        const int64_t seed_qc = 1024;
        ScopedTiming t(ix.timer_main, st);
        if (seeded && bounded) {
            sh.seed.ensure(sizeof(float) * (size_t)nq, sh.device);
            sh.cand.ensure(std::max(ncell * ((size_t)cap * 8 + 4), (size_t)std::min(nq, seed_qc) * sample * sizeof(float)),
                           sh.device);
            if (i8) {  // the queries' scales, residuals (the rerank's query term) and int8 image
                sh.qscale.ensure(sizeof(float) * (size_t)nq, sh.device);
                sh.qres.ensure(sizeof(float) * (size_t)nq, sh.device);
                if (i8_prep) {
                    launch_i8_query_prep(xq, nq, d, qn_launch ? sh.qn.get<float>() : nullptr, sh.qscale.get<float>(),
                                         sh.qres.get<float>(), 32 * W, sh.qimg.p, st);
                    qn_launch = false;
                } else {
                    launch_i8_row_scale(xq, nq, d, sh.qscale.get<float>(), sh.qres.get<float>(), st);
                    launch_i8_tile_rows(xq, sh.qscale.get<float>(), nq, d, 32 * W, sh.qimg.p, st);
                }
                qsc = sh.qscale.get<float>();
            } else {
                launch_b16_tile_rows(xq, nq, d, 32 * W, sh.qimg.p, st);
            }
            const size_t qtile_bytes = i8 ? flat_i8_img_bytes(32 * W, d, 32 * W) : flat_bf16_img_bytes(32 * W, d, 32 * W);
            for (int64_t c0 = 0; c0 < nq; c0 += seed_qc) {
                const int64_t cn = std::min(seed_qc, nq - c0);
                launch_flat_bf16_k64(static_cast<const char *>(sh.qimg.p) + (size_t)(c0 / (32 * W)) * qtile_bytes,
                                     qn ? qn + c0 : nullptr, cn, ximg, sh.xn.get<float>(), sample, nk, metric,
                                     (int)ceil_div(cn, 32 * W), (int)(sample / flat_bf16_tile_rows()), 1, 0, 1, nullptr,
                                     sh.cand.get<float>(), nullptr, nullptr, 0, false, true, st, qsc ? qsc + c0 : nullptr,
                                     xsc);
                launch_flat_keys_kth(sh.cand.get<float>(), (int)sample, cn, k, sh.seed.get<float>() + c0, st);
            }
        } else if (seeded) {
            const int64_t seed_rows = 65536;
            const int64_t stiles = seed_rows / flat_bf16_tile_rows();
            const int64_t snsplit = std::min<int64_t>(stiles, std::max<int64_t>(1, ceil_div(256, nqt)));
            const int64_t stps = ceil_div(stiles, snsplit);
            sh.seed.ensure(sizeof(float) * ((size_t)snsplit * nq * k * 2 + (size_t)nq), sh.device);
            float *spd = sh.seed.get<float>() + nq;
            int *spi = reinterpret_cast<int *>(spd + (size_t)snsplit * nq * k);
            launch_flat_bf16_topk(xq, qn, nq, sh.qimg.p, sh.xb16.p, sh.xn.get<float>(), seed_rows, d, metric, k,
                                  (int)ceil_div(stiles, stps), stps, spd, spi, nullptr, false, st);
            launch_flat_bf16_seed(spd, (int)ceil_div(stiles, stps), nq, k, sh.seed.get<float>(), st);
        }
        // bounded passes (64-dim K-step kernel, flat_b16k64.hip): every row with key ≤ the bound goes to a
        // per-(query, split) candidate buffer.  Pass 0 covers the first tiles of every split under the 16K-row
        // seed bound; after each pass the bound is re-merged from all candidates so far (the k-th best key over
        // every row scanned) and the next pass continues (flat_pass_plan: at 10M rows 4 passes over 5 / 20 / 98 /
        // 488 tiles per split, ≈ 8.5 candidates per query and split), no row scanned twice.  flat_cand_select keeps
        // each query's k best for the rerank.
        if (seeded && bounded) {
            static const bool dbg = std::getenv("HIPANN_FLAT_CAND_DEBUG") != nullptr;
            float *cd = sh.cand.get<float>();
            int *ci = reinterpret_cast<int *>(cd + ncell * cap);
            int *cn = ci + ncell * cap;
            float *bound = sh.seed.get<float>();
            for (size_t p = 0; p + 1 < pb.size(); ++p) {
                launch_flat_bf16_k64(sh.qimg.p, qn, nq, ximg, sh.xn.get<float>(), sh.n, nk, metric, (int)nqt,
                                     (int)nsplit, tps, pb[p], pb[p + 1], bound, cd, ci, cn, cap, p > 0, false, st, qsc,
                                     xsc);
                if (p + 2 < pb.size()) launch_flat_cand_bound(cd, cn, (int)nsplit, cap, nq, k, bound, st);
            }
            sh.nflag.ensure(sizeof(int), sh.device);
            sh.flagged.ensure(sizeof(int) * (size_t)nq, sh.device);
            HIPANN_CHECK(hipMemsetAsync(sh.nflag.p, 0, sizeof(int), st));
            // overflowed queries are flagged here, ahead of the rerank's own flags (the fallback re-runs both)
            launch_flat_cand_select(cd, ci, cn, (int)nsplit, cap, nq, k, sh.part_d.get<float>(), sh.part_i.get<int>(),
                                    sh.nflag.get<int>(), sh.flagged.get<int>(), st);
            if (dbg) {
                std::vector<int> hn(ncell);
                std::vector<float> hb((size_t)nq);
                HIPANN_CHECK(hipMemcpyAsync(hn.data(), cn, sizeof(int) * ncell, hipMemcpyDeviceToHost, st));
                HIPANN_CHECK(hipMemcpyAsync(hb.data(), bound, sizeof(float) * nq, hipMemcpyDeviceToHost, st));
                HIPANN_CHECK(hipStreamSynchronize(st));
                long long tot = 0;
                int mx = 0;
                for (int v : hn) { tot += v; mx = std::max(mx, v); }
                std::fprintf(stderr, "hipann flat cand: nsplit %lld tps %lld passes %zu pass0 %lld cap %d mean %.2f max %d bound[0] %g\n",
                             (long long)nsplit, (long long)tps, pb.size() - 1, (long long)pb[1], cap, (double)tot / (double)ncell, mx,
                             (double)hb[0]);
            }
            cr_d = cd;
            cr_i = ci;
            cr_n = cn;
            cr_nsplit = (int)nsplit;
            cr_cap = cap;
            cr_bound = bound;
            nsplit = 1;
            flags_ready = true;
        } else {
            launch_flat_bf16_topk(xq, qn, nq, sh.qimg.p, sh.xb16.p, sh.xn.get<float>(), sh.n, d, metric, k,
                                  (int)nsplit, tps, sh.part_d.get<float>(), sh.part_i.get<int>(),
                                  seeded ? sh.seed.get<float>() : nullptr, seeded, st);
        }
    } else {
        const int64_t nqt = ceil_div(nq, 128);
        const int64_t ntiles = ceil_div(sh.n, 128);
        // ≈2048 blocks; small tables (an IVF coarse quantizer: 1024 centroids = 8 tiles) go down to one
        // column tile per block rather than leaving CUs idle
        nsplit = std::max<int64_t>(1, ceil_div(2048, nqt));
        nsplit = std::min<int64_t>(nsplit, ntiles);
        if (nsplit >= 8) nsplit = nsplit / 8 * 8;
        const int64_t tps = ceil_div(ntiles, nsplit);
        nsplit = ceil_div(ntiles, tps);
        HIPANN_REQUIRE(nqt * nsplit < (int64_t)0x7fffffff, "grid too large");
        sh.part_d.ensure((size_t)nsplit * nq * k * sizeof(float), sh.device);
        sh.part_i.ensure((size_t)nsplit * nq * k * sizeof(int), sh.device);
        ScopedTiming t(ix.timer_main, st);
        if (form == kFlatFp32) {
            launch_flat_gemm_topk(xq, qn, nq, sh.xb, sh.xn.get<float>(), sh.n, d, metric, k, (int)nsplit, tps,
                                  sh.part_d.get<float>(), sh.part_i.get<int>(), st);
        } else {
            const int np = form == kFlatSplit3 ? 3 : 2;
            sh.qsplit.ensure(flat_bf_qsplit_bytes(nq, d, np), sh.device);
            launch_flat_gemm_topk_bf(np, xq, qn, nq, sh.qsplit.get<void>(), sh.xb, sh.xn.get<float>(), sh.n, d, metric,
                                     k, (int)nsplit, tps, sh.part_d.get<float>(), sh.part_i.get<int>(), exact ? 1 : 0,
                                     st);
        }
    }
    if (!exact) {
        ScopedTiming t(ix.timer_merge, st);
        launch_merge_parts<int>(sh.part_d.get<float>(), sh.part_i.get<int>(), (int)nsplit, nq, k, kout, sh.label_offset,
                                1.f, out_sign, D, I, st);
        return;
    }
    // exact form: merge each query's nsplit lists to the 16 best scan keys, recompute those rows in the
    // direct form, bound-check (ivf_rerank_topk, slot lists query-major); flagged queries re-run on split3
    if (!flags_ready) {
        sh.nflag.ensure(sizeof(int), sh.device);
        sh.flagged.ensure(sizeof(int) * (size_t)nq, sh.device);
        HIPANN_CHECK(hipMemsetAsync(sh.nflag.p, 0, sizeof(int), st));
    }
    {
        ScopedTiming t(ix.timer_merge, st);
        // (int8: the row term and each query's own residual from the int8 images; qres makes the rerank read them)
        launch_ivf_rerank(sh.part_d.get<float>(), sh.part_i.get<int>(), nullptr, (int)nsplit, nq, k, kout, metric, xq,
                          sh.xb, d, nullptr, sh.n, sh.label_offset, xmax2, D, I, sh.nflag.get<int>(),
                          sh.flagged.get<int>(), st, kSplit2Eps, form == kFlatBf16Exact || i8 ? rxmax : -1.f,
                          i8 ? sh.qres.get<float>() : nullptr);
    }
    pend = FlatPending{};
    pend.kind = FlatPending::kExact;
    pend.nq = nq;
    pend.xq = xq;
    pend.k = k_user;
    pend.kout = kout;
    pend.D = D;
    pend.I = I;
    pend.cr_d = cr_d;
    pend.cr_bound = cr_bound;
    pend.cr_i = cr_i;
    pend.cr_n = cr_n;
    pend.cr_nsplit = cr_nsplit;
    pend.cr_cap = cr_cap;
    pend.xmax2 = xmax2;
    pend.rxmax = rxmax;
    pend.i8 = i8;
    flag_readback(sh, st);
}

// The second half of a shard search, once the host has synchronised with the launch phase's stream (its flag
// count read back into sh.h_nflag): nothing to do unless the exact form's bound check flagged queries.  Flagged
// queries are rare (0 on every benchmark batch); their re-runs are synchronous.
void flat_shard_finish(FlatIndex &ix, FlatShard &sh, const FlatPending &pend, hipStream_t st) {
    if (pend.kind == FlatPending::kNone) return;
    int nf = *sh.h_nflag.get<int>();
    if (nf <= 0) return;
    DeviceGuard g(sh.device);
    const int d = ix.d, metric = ix.metric;
    const int kout = pend.kout;
    const float *xq = pend.xq;
    float *D = pend.D;
    int64_t *I = pend.I;
    int *fl = sh.flagged.get<int>();
    int rerun_form = kFlatSplit3;
    if (pend.kind == FlatPending::kSmallI8) {
        rerun_form = kFlatFp32;
    } else if (pend.cr_d) {
        const float *cr_d = pend.cr_d, *cr_bound = pend.cr_bound;
        const int *cr_i = pend.cr_i, *cr_n = pend.cr_n;
        const int cr_nsplit = pend.cr_nsplit, cr_cap = pend.cr_cap;
        const float xmax2 = pend.xmax2, rxmax = pend.rxmax;
        const bool i8 = pend.i8;
        // bounded passes: rerank each flagged query over all its buffered candidates, certified against the pass
        // bound (launch_flat_cand_rerank); only what that cannot certify re-runs on SPLIT3
        const int P = flat_cand_rerank_parts(cr_nsplit);
        sh.crd.ensure(sizeof(float) * (size_t)nf * P * kout, sh.device);
        sh.cri.ensure(sizeof(long long) * (size_t)nf * P * kout, sh.device);
        sh.covf.ensure(sizeof(int) * (size_t)nf * P, sh.device);
        sh.nflag2.ensure(sizeof(int), sh.device);
        sh.flagged2.ensure(sizeof(int) * (size_t)nf, sh.device);
        HIPANN_CHECK(hipMemsetAsync(sh.nflag2.p, 0, sizeof(int), st));
        static const bool dbg = std::getenv("HIPANN_FLAT_CAND_DEBUG") != nullptr;
        if (dbg) sh.tmpnorm.ensure(sizeof(float) * 4 * (size_t)nf, sh.device);
        {
            ScopedTiming t(ix.timer_merge, st);
            launch_flat_cand_rerank(fl, nf, cr_d, cr_i, cr_n, cr_nsplit, cr_cap, cr_bound, xq, sh.xb, d, sh.n,
                                    sh.label_offset, xmax2, rxmax, metric, kout, sh.crd.get<float>(),
                                    sh.cri.get<long long>(), sh.covf.get<int>(), D, I, sh.nflag2.get<int>(),
                                    sh.flagged2.get<int>(), st, dbg ? sh.tmpnorm.get<float>() : nullptr,
                                    i8 ? sh.qres.get<float>() : nullptr);
        }
        ix.cand_reranked += nf;
        const int nf1 = nf;
        HIPANN_CHECK(hipMemcpyAsync(&nf, sh.nflag2.p, sizeof(int), hipMemcpyDeviceToHost, st));
        HIPANN_CHECK(hipStreamSynchronize(st));
        ++ix.host_syncs;
        if (dbg) {
            std::vector<float> h((size_t)nf1 * 4);
            HIPANN_CHECK(hipMemcpy(h.data(), sh.tmpnorm.p, h.size() * sizeof(float), hipMemcpyDeviceToHost));
            std::fprintf(stderr, "hipann flat flagged %d -> %d after the candidate rerank\n", nf1, nf);
            for (int j = 0; j < nf1 && j < 8; ++j)
                std::fprintf(stderr, "  overflow %g  dk %g  T %g  E %g\n", h[4 * j], h[4 * j + 1], h[4 * j + 2], h[4 * j + 3]);
        }
        if (nf <= 0) return;
        fl = sh.flagged2.get<int>();
    }
    ix.rerank_fallbacks += nf;
    sh.fq.ensure(sizeof(float) * (size_t)nf * d, sh.device);
    sh.fD.ensure(sizeof(float) * (size_t)nf * kout, sh.device);
    sh.fI.ensure(sizeof(int64_t) * (size_t)nf * kout, sh.device);
    launch_ivf_gather_queries(xq, fl, nf, d, sh.fq.get<float>(), st);
    {
        TimerPause p0(ix.timer_main), p1(ix.timer_merge);
        flat_shard_search(ix, sh, nf, sh.fq.get<float>(), pend.k, kout, sh.fD.get<float>(), sh.fI.get<int64_t>(), st,
                          rerun_form);
    }
    launch_ivf_scatter_results(sh.fD.get<float>(), sh.fI.get<int64_t>(), fl, nf, kout, D, I, st);
}

void flat_shard_search(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                       int64_t *I, hipStream_t st, int form_override, FlatPending *pend) {
    RoctxRange r_all("hipann.flat.search_shard");
    FlatPending local;
    flat_shard_launch(ix, sh, nq, xq, k, kout, D, I, st, form_override, pend ? *pend : local);
    if (pend || local.kind == FlatPending::kNone) return;
    wait_posted(sh.h_nflag.get<unsigned>() + 1, sh.flag_seq, st);  // the flag count's token: the launch phase is done
    ++ix.host_syncs;
    flat_shard_finish(ix, sh, local, st);
}

}  // namespace hipann

// ================================================================================================
extern "C" {

int hipann_available(void) {
    try {
        if (device_count() <= 0) return 0;
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 0;
        return std::strstr(p.gcnArchName, "gfx950") ? 1 : 0;
    } catch (...) {
        return 0;
    }
}

int hipann_device_count(void) { return device_count(); }

int hipann_peer_access(void *h, int *state, int cap, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        std::lock_guard<std::mutex> lk(ix->mu);
        // single-device handles (the _device creates) carry no list: one shard, on its own device
        const std::vector<int> one{2};
        const std::vector<int> &pv = ix->peer.empty() ? one : ix->peer;
        const int n = (int)pv.size();
        HIPANN_REQUIRE(!state || cap >= n, "state buffer too small");
        if (state) for (int i = 0; i < n; ++i) state[i] = pv[(size_t)i];
        return n;
    });
}

int hipann_device_info(char *buf, int buf_len) {
    try {
        std::string s;
        const int n = device_count();
        if (n <= 0) s = "HIP: no device available";
        else {
            hipDeviceProp_t p;
            HIPANN_CHECK(hipGetDeviceProperties(&p, 0));
            char tmp[512];
            std::snprintf(tmp, sizeof tmp, "%s (%s, %d CUs, %.0f GB HBM) x%d", p.name, p.gcnArchName,
                          p.multiProcessorCount, (double)p.totalGlobalMem / 1e9, n);
            s = tmp;
        }
        set_err(buf, buf_len, s.c_str());
        return (int)s.size();
    } catch (...) {
        return -1;
    }
}

void *hipann_flat_create(int d, int metric, const float *xb, int64_t n, const int *devices, int ndev, char *eb,
                         int el) {
    return guard_ptr(eb, el, [&]() -> void * {
        require_device();
        HIPANN_REQUIRE(d > 0, "d must be > 0");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 (L2) or 1 (IP)");
        HIPANN_REQUIRE(n >= 0 && (n == 0 || xb), "invalid vectors");
        auto devs = device_list(devices, ndev);
        auto ix = std::make_unique<FlatIndex>();
        ix->d = d;
        ix->metric = metric;
        const int64_t per = ceil_div(std::max<int64_t>(n, 1), (int64_t)devs.size());
        int64_t off = 0;
        for (size_t i = 0; i < devs.size(); ++i) {
            auto sh = std::make_unique<FlatShard>();
            sh->device = devs[i];
            sh->stream = make_stream(devs[i]);
            sh->label_offset = off;
            const int64_t cnt = std::min<int64_t>(per, n - off);
            if (cnt > 0) shard_append(*sh, d, metric, xb + off * (int64_t)d, nullptr, cnt);
            off += std::max<int64_t>(cnt, 0);
            ix->shards.push_back(std::move(sh));
        }
        ix->peer = enable_peer_access(devs);
        return ix.release();
    });
}

int hipann_flat_add(void *h, const float *xb, int64_t n, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::Flat, "not a Flat index");
        auto *fx = static_cast<FlatIndex *>(ix);
        std::lock_guard<std::mutex> lk(fx->mu);
        HIPANN_REQUIRE(n >= 0 && (n == 0 || xb), "invalid vectors");
        // appended rows go to the last shard (labels stay contiguous)
        auto &sh = *fx->shards.back();
        shard_append(sh, fx->d, fx->metric, xb, nullptr, n);
        return 0;
    });
}

static int flat_search_host(FlatIndex &ix, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I) {
    HIPANN_REQUIRE(k > 0, "k must be > 0");
    HIPANN_REQUIRE(k <= HIPANN_MAX_K, "k larger than HIPANN_MAX_K");
    HIPANN_REQUIRE(nq >= 0 && (nq == 0 || (xq && D && I)), "invalid arguments");
    const float pad = ix.metric == kIP ? -__builtin_inff() : __builtin_inff();
    const int64_t ntot = ix.ntotal();
    if (nq == 0) return 0;
    if (ntot == 0) {
        for (int64_t i = 0; i < nq * k; ++i) { D[i] = pad; I[i] = -1; }
        return 0;
    }
    const int keff = (int)std::min<int64_t>(k, ntot);
    const int kout = (int)k;
    const size_t qbytes = (size_t)nq * ix.d * sizeof(float);
    ix.h_q.ensure(qbytes);
    std::memcpy(ix.h_q.p, xq, qbytes);
    const size_t ob = (size_t)nq * kout;
    const int np = (int)ix.shards.size();
    // Launch phase: every shard's search on its own stream (devices run concurrently), no host wait.  The exact
    // forms' flag counts travel to pinned host words with the results (flat_shard_finish reads them).
    std::vector<FlatPending> pend((size_t)np);
    for (int p = 0; p < np; ++p) {
        FlatShard &sh = *ix.shards[p];
        DeviceGuard g(sh.device);
        sh.q.ensure(qbytes, sh.device);
        sh.out_d.ensure(ob * sizeof(float), sh.device);
        sh.out_i.ensure(ob * sizeof(int64_t), sh.device);
        FenceScope fs(sh.fence, sh.stream, sh.device);
        if (qbytes <= kKernelCopyMax) launch_copy_words(host_device_ptr(ix.h_q.p), sh.q.p, qbytes, sh.stream);
        else HIPANN_CHECK(hipMemcpyAsync(sh.q.p, ix.h_q.p, qbytes, hipMemcpyHostToDevice, sh.stream));
        flat_shard_search(ix, sh, nq, sh.q.get<float>(), keff, kout, sh.out_d.get<float>(), sh.out_i.get<int64_t>(),
                          sh.stream, -1, &pend[(size_t)p]);
        if (np > 1) {
            if (!sh.done) HIPANN_CHECK(hipEventCreateWithFlags(&sh.done, hipEventDisableTiming));
            HIPANN_CHECK(hipEventRecord(sh.done, sh.stream));
        }
    }
    ix.h_d.ensure(ob * sizeof(float));
    ix.h_i.ensure(ob * sizeof(int64_t));
    FlatShard &s0 = *ix.shards[0];
    // Completion: results (merged on shard 0's device when sharded) to the host, ONE host synchronisation — which
    // also covers every shard's flag count.  Only if a shard flagged queries: its re-runs, then the results again.
    auto deliver = [&]() {
        if (np == 1) {
            DeviceGuard g(s0.device);
            if (ob * sizeof(int64_t) <= kKernelCopyMax) {
                launch_copy_words(s0.out_d.p, host_device_ptr(ix.h_d.p), ob * sizeof(float), s0.stream);
                launch_copy_words(s0.out_i.p, host_device_ptr(ix.h_i.p), ob * sizeof(int64_t), s0.stream);
            } else {
                HIPANN_CHECK(hipMemcpyAsync(ix.h_d.p, s0.out_d.p, ob * sizeof(float), hipMemcpyDeviceToHost, s0.stream));
                HIPANN_CHECK(hipMemcpyAsync(ix.h_i.p, s0.out_i.p, ob * sizeof(int64_t), hipMemcpyDeviceToHost, s0.stream));
            }
        } else {
            // gather the per-device partial top-k onto shard 0's device (shard 0's stream waits for each shard's
            // launch phase on the device, not the host), then one device merge
            DeviceGuard g(s0.device);
            ix.gather_d.ensure(ob * np * sizeof(float), s0.device);
            ix.gather_i.ensure(ob * np * sizeof(int64_t), s0.device);
            ix.merged_d.ensure(ob * sizeof(float), s0.device);
            ix.merged_i.ensure(ob * sizeof(int64_t), s0.device);
            for (int p = 0; p < np; ++p) {
                FlatShard &sh = *ix.shards[p];
                if (p > 0) HIPANN_CHECK(hipStreamWaitEvent(s0.stream, sh.done, 0));
                HIPANN_CHECK(hipMemcpyPeerAsync(ix.gather_d.get<float>() + p * ob, s0.device, sh.out_d.p, sh.device,
                                                ob * sizeof(float), s0.stream));
                HIPANN_CHECK(hipMemcpyPeerAsync(ix.gather_i.get<int64_t>() + p * ob, s0.device, sh.out_i.p, sh.device,
                                                ob * sizeof(int64_t), s0.stream));
            }
            const float sign = ix.metric == kIP ? -1.f : 1.f;
            launch_merge_parts<long long>(ix.gather_d.get<float>(), ix.gather_i.get<long long>(), np, nq, kout, kout, 0,
                                          sign, sign, ix.merged_d.get<float>(), ix.merged_i.get<int64_t>(), s0.stream);
            HIPANN_CHECK(hipMemcpyAsync(ix.h_d.p, ix.merged_d.p, ob * sizeof(float), hipMemcpyDeviceToHost, s0.stream));
            HIPANN_CHECK(hipMemcpyAsync(ix.h_i.p, ix.merged_i.p, ob * sizeof(int64_t), hipMemcpyDeviceToHost, s0.stream));
        }
        DeviceGuard g(s0.device);
        HIPANN_CHECK(hipStreamSynchronize(s0.stream));
        ++ix.host_syncs;
    };
    deliver();
    bool rerun = false;
    for (int p = 0; p < np; ++p) {
        FlatShard &sh = *ix.shards[p];
        if (pend[(size_t)p].kind == FlatPending::kNone || *sh.h_nflag.get<int>() <= 0) continue;
        FenceScope fs(sh.fence, sh.stream, sh.device);
        flat_shard_finish(ix, sh, pend[(size_t)p], sh.stream);
        if (np > 1) {
            DeviceGuard g(sh.device);
            HIPANN_CHECK(hipEventRecord(sh.done, sh.stream));
        }
        rerun = true;
    }
    if (rerun) deliver();
    std::memcpy(D, ix.h_d.p, ob * sizeof(float));
    std::memcpy(I, ix.h_i.p, ob * sizeof(int64_t));
    return 0;
}

int hipann_flat_search(void *h, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::Flat, "not a Flat index");
        auto *fx = static_cast<FlatIndex *>(ix);
        std::lock_guard<std::mutex> lk(fx->mu);
        return flat_search_host(*fx, nq, xq, k, D, I);
    });
}

int hipann_flat_reconstruct(void *h, int64_t key, float *out, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h && out, "null argument");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::Flat, "not a Flat index");
        auto *fx = static_cast<FlatIndex *>(ix);
        std::lock_guard<std::mutex> lk(fx->mu);
        for (auto &shp : fx->shards) {
            FlatShard &sh = *shp;
            if (key >= sh.label_offset && key < sh.label_offset + sh.n) {
                DeviceGuard g(sh.device);
                HIPANN_CHECK(hipMemcpyAsync(out, sh.xb + (key - sh.label_offset) * fx->d, (size_t)fx->d * sizeof(float),
                                            hipMemcpyDeviceToHost, sh.stream));
                HIPANN_CHECK(hipStreamSynchronize(sh.stream));
                return 0;
            }
        }
        throw HipError("hipann: reconstruct key out of range");
    });
}

int hipann_flat_reconstruct_n(void *h, int64_t i0, int64_t n, float *out, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h && (n == 0 || out), "null argument");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::Flat, "not a Flat index");
        auto *fx = static_cast<FlatIndex *>(ix);
        std::lock_guard<std::mutex> lk(fx->mu);
        HIPANN_REQUIRE(i0 >= 0 && n >= 0 && i0 + n <= fx->ntotal(), "hipann: reconstruct_n range out of bounds");
        for (auto &shp : fx->shards) {  // shards hold contiguous label ranges
            FlatShard &sh = *shp;
            const int64_t lo = std::max(i0, sh.label_offset), hi = std::min(i0 + n, sh.label_offset + sh.n);
            if (lo >= hi) continue;
            DeviceGuard g(sh.device);
            HIPANN_CHECK(hipMemcpyAsync(out + (lo - i0) * fx->d, sh.xb + (lo - sh.label_offset) * fx->d,
                                        sizeof(float) * (size_t)(hi - lo) * fx->d, hipMemcpyDeviceToHost, sh.stream));
            HIPANN_CHECK(hipStreamSynchronize(sh.stream));
        }
        return 0;
    });
}

void *hipann_flat_create_device(int d, int metric, const float *xb_dev, int64_t n, int device, int copy,
                                int64_t label_offset, char *eb, int el) {
    return guard_ptr(eb, el, [&]() -> void * {
        require_device();
        HIPANN_REQUIRE(d > 0, "d must be > 0");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 (L2) or 1 (IP)");
        HIPANN_REQUIRE(device >= 0 && device < device_count(), "invalid device");
        HIPANN_REQUIRE(n >= 0 && (n == 0 || xb_dev), "invalid vectors");
        {   // the caller's writes to xb_dev may still be in flight on any of its streams
            DeviceGuard g(device);
            HIPANN_CHECK(hipDeviceSynchronize());
        }
        auto ix = std::make_unique<FlatIndex>();
        ix->d = d;
        ix->metric = metric;
        auto sh = std::make_unique<FlatShard>();
        sh->device = device;
        sh->stream = make_stream(device);
        sh->label_offset = label_offset;
        if (copy) {
            shard_append(*sh, d, metric, nullptr, xb_dev, n);
        } else {
            DeviceGuard g(device);
            sh->xb = const_cast<float *>(xb_dev);
            sh->owns = false;
            sh->n = n;
            sh->cap = n;
            if (metric == kL2 && n > 0) {
                sh->xn.ensure((size_t)n * sizeof(float), device);
                launch_row_norms(sh->xb, n, d, sh->xn.get<float>(), sh->stream);
                HIPANN_CHECK(hipStreamSynchronize(sh->stream));
            }
        }
        ix->shards.push_back(std::move(sh));
        return ix.release();
    });
}

int hipann_flat_search_device(void *h, int64_t nq, const float *xq_dev, int64_t k, float *D_dev, int64_t *I_dev,
                              void *stream, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::Flat, "not a Flat index");
        auto *fx = static_cast<FlatIndex *>(ix);
        std::lock_guard<std::mutex> lk(fx->mu);
        HIPANN_REQUIRE(fx->shards.size() == 1, "device search needs a single-device index");
        HIPANN_REQUIRE(k > 0 && k <= HIPANN_MAX_K, "k out of range");
        FlatShard &sh = *fx->shards[0];
        hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = the default (null) stream
        const int keff = (int)std::min<int64_t>(k, std::max<int64_t>(sh.n, 1));
        FenceScope fs(sh.fence, st, sh.device);  // the previous call's kernels may still use this shard's scratch
        flat_shard_search(*fx, sh, nq, xq_dev, keff, (int)k, D_dev, I_dev, st);
        return 0;
    });
}

int hipann_merge_topk_device(int metric, int nparts, int64_t nq, int64_t k, const float *D_parts,
                             const int64_t *I_parts, float *D_out, int64_t *I_out, void *stream, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        require_device();
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "bad metric");
        HIPANN_REQUIRE(k > 0 && k <= HIPANN_MAX_K && nparts >= 0, "bad arguments");
        const float sign = metric == kIP ? -1.f : 1.f;
        launch_merge_parts<long long>(D_parts, reinterpret_cast<const long long *>(I_parts), nparts, nq, (int)k, (int)k,
                                      0, sign, sign, D_out, I_out, static_cast<hipStream_t>(stream));
        return 0;
    });
}

int hipann_merge_topk_packed_device(int metric, int nparts, int64_t nq, int64_t k, const void *parts,
                                    int64_t part_bytes, float *D_out, int64_t *I_out, void *stream, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        require_device();
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "bad metric");
        HIPANN_REQUIRE(k > 0 && k <= HIPANN_MAX_K && nparts >= 0, "bad arguments");
        HIPANN_REQUIRE(part_bytes % 8 == 0 && part_bytes >= nq * k * 12, "part_bytes too small / misaligned");
        const float sign = metric == kIP ? -1.f : 1.f;
        const char *base = static_cast<const char *>(parts);
        // part p: [labels int64 nq*k][distances fp32 nq*k] at base + p * part_bytes
        launch_merge_parts<long long>(reinterpret_cast<const float *>(base + nq * k * 8),
                                      reinterpret_cast<const long long *>(base), nparts, nq, (int)k, (int)k, 0, sign,
                                      sign, D_out, I_out, static_cast<hipStream_t>(stream), part_bytes / 4,
                                      part_bytes / 8);
        return 0;
    });
}

int64_t hipann_ntotal(void *h) { return h ? static_cast<IndexBase *>(h)->ntotal() : -1; }
int hipann_dim(void *h) { return h ? static_cast<IndexBase *>(h)->d : -1; }
int hipann_metric(void *h) { return h ? static_cast<IndexBase *>(h)->metric : -1; }
int64_t hipann_memory_bytes(void *h) { return h ? static_cast<IndexBase *>(h)->memory_bytes() : -1; }

int hipann_flat_set_form(void *h, int form) {
    if (!h || form < kFlatFp32 || form > kFlatI8Exact) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::Flat) return -1;
    auto *fx = static_cast<FlatIndex *>(ix);
    std::lock_guard<std::mutex> lk(fx->mu);
    fx->form = form;
    return 0;
}

int64_t hipann_flat_rerank_fallbacks(void *h) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::Flat) return -1;
    return static_cast<FlatIndex *>(ix)->rerank_fallbacks;
}

int64_t hipann_flat_host_syncs(void *h) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::Flat) return -1;
    std::lock_guard<std::mutex> lk(ix->mu);
    return static_cast<FlatIndex *>(ix)->host_syncs;
}

int hipann_last_search_path(void *h, int *form, int *filter_k, int *sublists) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    std::lock_guard<std::mutex> lk(ix->mu);
    if (form) *form = ix->last_form;
    if (filter_k) *filter_k = ix->last_kfilt;
    if (sublists) *sublists = ix->last_sublists;
    return 0;
}

int hipann_flat_get_form(void *h) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::Flat) return -1;
    return static_cast<FlatIndex *>(ix)->form;
}

void hipann_free(void *h) {
    if (!h) return;
    try {
        delete static_cast<IndexBase *>(h);
    } catch (...) {
    }
}

int hipann_set_kernel_timing(void *h, int on) {
    try {
        if (!h) return -1;
        auto *ix = static_cast<IndexBase *>(h);
        std::lock_guard<std::mutex> lk(ix->mu);
        ix->timer_main.reset(on != 0, 0);
        ix->timer_merge.reset(on != 0, 0);
        return 0;
    } catch (...) {
        return -1;
    }
}

double hipann_last_kernel_ms(void *h, int which) {
    try {
        if (!h) return 0.0;
        auto *ix = static_cast<IndexBase *>(h);
        std::lock_guard<std::mutex> lk(ix->mu);
        return which == 0 ? ix->timer_main.average_ms() : ix->timer_merge.average_ms();
    } catch (...) {
        return 0.0;
    }
}

}  // extern "C"
