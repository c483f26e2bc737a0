// ivf.cpp — IVFFlat part of the C ABI (include/hip_ann.h).
//
// Mirrors index_cpu_to_metal_ivf (faiss-metal/src/MetalIndexIVFFlat.mm:283-326: centroids, per-list
// ids and raw fp32 codes copied out of a FAISS IndexIVFFlat; nprobe taken from the CPU index) and
// MetalIndexIVFFlat::search (:122-256: k <= 0 throws, empty → (±inf, −1) pads, ids remapped to the
// stored labels).  The parity target is FAISS CPU IndexIVFFlat::search: coarse search
// with nprobe = min(nprobe, nlist), lists scanned with direct distances.
#include "../../include/hip_ann.h"
#include "ivf.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <numeric>

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

hipStream_t make_stream(int dev) {
    DeviceGuard g(dev);
    hipStream_t s;
    HIPANN_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}

// The search-time coarse step's key GEMM on the bf16 matrix cores (flat_keys_bf3: three-term split, fp32-level
// keys; HIPANN_COARSE_BF3=0 keeps the fp32 matrix cores, A/B).  List assignment (add / append) keeps fp32.
static bool coarse_bf3() {
    static const bool v = [] { const char *e = std::getenv("HIPANN_COARSE_BF3"); return !e || std::atoi(e) != 0; }();
    return v;
}
struct CoarseKeysScope {
    FlatShard &s;
    explicit CoarseKeysScope(FlatShard &x) : s(x) { s.keys_bf3 = coarse_bf3(); }
    ~CoarseKeysScope() { s.keys_bf3 = false; }
};

// Borrowed-centroid coarse quantizer on the shard's device.
std::unique_ptr<FlatIndex> make_quantizer(int d, int metric, const float *cen, int nlist, int device,
                                          hipStream_t stream) {
    auto q = std::make_unique<FlatIndex>();
    q->form = kFlatFp32;  // coarse assignment stays on exact fp32 products
    q->d = d;
    q->metric = metric;
    auto sh = std::make_unique<FlatShard>();
    sh->device = device;
    sh->stream = nullptr;  // searches run on the IVF shard's stream
    sh->xb = const_cast<float *>(cen);
    sh->owns = false;
    sh->n = nlist;
    sh->cap = nlist;
    if (metric == kL2) {
        DeviceGuard g(device);
        sh->xn.ensure((size_t)nlist * sizeof(float), device);
        launch_row_norms(cen, nlist, d, sh->xn.get<float>(), stream);
        HIPANN_CHECK(hipStreamSynchronize(stream));
    }
    q->shards.push_back(std::move(sh));
    return q;
}

// off: physical list starts (nlist + 1; list l owns rows [off[l], off[l+1])), len: live rows per list (≤ capacity).
void upload_list_meta(IvfShard &sh, const std::vector<int64_t> &off, const std::vector<int64_t> &len, int nlist) {
    DeviceGuard g(sh.device);
    std::vector<int> hl(nlist);
    int64_t maxlen = 0, live = 0;
    for (int l = 0; l < nlist; ++l) {
        HIPANN_REQUIRE(len[l] >= 0 && len[l] <= off[l + 1] - off[l], "list length exceeds its capacity");
        HIPANN_REQUIRE(len[l] < (int64_t)0x7fffffff, "inverted list longer than 2^31-1 rows");
        hl[l] = (int)len[l];
        maxlen = std::max<int64_t>(maxlen, len[l]);
        live += len[l];
    }
    sh.max_nch = (int)std::max<int64_t>(1, ceil_div(maxlen, ivf_chunk_rows()));
    sh.h_off = off;
    sh.h_len = len;
    sh.n = off[nlist];
    sh.live = live;
    sh.list_off.ensure(sizeof(int64_t) * (nlist + 1), sh.device);
    sh.list_len.ensure(sizeof(int) * nlist, sh.device);
    HIPANN_CHECK(hipMemcpyAsync(sh.list_off.p, off.data(), sizeof(int64_t) * (nlist + 1), hipMemcpyHostToDevice,
                                sh.stream));
    HIPANN_CHECK(hipMemcpyAsync(sh.list_len.p, hl.data(), sizeof(int) * nlist, hipMemcpyHostToDevice, sh.stream));
    HIPANN_CHECK(hipStreamSynchronize(sh.stream));
}

std::vector<int64_t> dense_lengths(const std::vector<int64_t> &off, int nlist) {
    std::vector<int64_t> len(nlist);
    for (int l = 0; l < nlist; ++l) len[l] = off[l + 1] - off[l];
    return len;
}

// 32-row pass offsets of every list (the tiled copies' layout); returns the total pass count.
int64_t ensure_tpass(IvfShard &sh, int nlist, hipStream_t st) {
    std::vector<int64_t> tp(nlist + 1, 0);
    for (int l = 0; l < nlist; ++l) tp[l + 1] = tp[l] + ceil_div(sh.h_off[l + 1] - sh.h_off[l], 32);
    if (!sh.tpass_off.p) {
        sh.tpass_off.ensure(sizeof(int64_t) * (nlist + 1), sh.device);
        HIPANN_CHECK(hipMemcpyAsync(sh.tpass_off.p, tp.data(), sizeof(int64_t) * (nlist + 1), hipMemcpyHostToDevice, st));
        HIPANN_CHECK(hipStreamSynchronize(st));  // tp (host) is released on return
    }
    return tp[nlist];
}

// The MFMA scan's tiled copy of the codes (built once, at the first search that uses it).
void ensure_tiled_codes(IvfShard &sh, int d, int nlist, hipStream_t st) {
    if (sh.codes_t.p || sh.n == 0) return;
    const int64_t np = ensure_tpass(sh, nlist, st);
    const int64_t pf = ivf_mfma_pass_floats(d);
    sh.codes_t.ensure(sizeof(float) * (size_t)std::max<int64_t>(np, 1) * pf, sh.device);
    launch_ivf_tile_codes(sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(), sh.tpass_off.get<int64_t>(), nlist,
                          np, d, sh.codes_t.get<float>(), st);
    HIPANN_CHECK(hipStreamSynchronize(st));
}

// kFormHalfExact: the tiled fp16 image of x·s, s = 2^half_es with max|x| = f·2^e, f ∈ [½, 1), half_es =
// 14 − e (every scaled element < 2^14), and the largest row residual ‖x − x̂/s‖ (built once).  Codes
// with a non-finite entry or a scale outside 2^±100 leave the form unsupported (the search then takes
// kFormSplit2Exact).  Returns whether the image is usable.
bool ensure_half_codes(IvfShard &sh, int d, int nlist, hipStream_t st) {
    if (sh.half_state != 0) return sh.half_state > 0;
    if (sh.n == 0) return false;  // nothing to scan (and nothing to measure); retried after an add
    sh.nflag.ensure(sizeof(int), sh.device);
    unsigned bits = 0;
    launch_ivf_max_abs(sh.codes, sh.n * (int64_t)d, sh.nflag.get<unsigned>(), st);
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    float mx;
    std::memcpy(&mx, &bits, sizeof(mx));
    int e = 0;
    if (bits != 0 && bits < 0x7f800000u) (void)std::frexp(mx, &e);
    if (bits >= 0x7f800000u || e < -100 || e > 100) {
        sh.half_state = -1;
        return false;
    }
    sh.half_es = 14 - e;
    const float scale = std::ldexp(1.f, sh.half_es);
    const int64_t np = ensure_tpass(sh, nlist, st);
    sh.codes_h.ensure((size_t)std::max<int64_t>(np, 1) * (size_t)ivf_half_pass_bytes(d), sh.device);
    launch_ivf_tile_half(sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(), sh.tpass_off.get<int64_t>(), nlist,
                         np, d, scale, sh.codes_h.p, st);
    launch_ivf_half_residual(sh.codes, sh.n, d, scale, sh.nflag.get<unsigned>(), st);
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    float r2;
    std::memcpy(&r2, &bits, sizeof(r2));
    sh.half_rxmax = std::sqrt(r2) * 1.0001f;  // fp32 sum of d exact squares: relative error ≪ 1e-4
    sh.half_state = 1;
    return true;
}

// kFormI8Exact: the tiled int8 image (one scale per row, ivf_mfma.hip) and its largest row residual, built at the
// first search that needs them (and again after an append: appends release it)
bool ensure_i8_codes(IvfShard &sh, int d, int nlist, hipStream_t st) {
    if (sh.i8_state != 0) return sh.i8_state > 0;
    if (sh.n == 0) return false;
    const int64_t np = ensure_tpass(sh, nlist, st);
    sh.codes_i8.ensure((size_t)std::max<int64_t>(np, 1) * (size_t)ivf_i8_pass_bytes(d), sh.device);
    sh.xs8.ensure(sizeof(float) * (size_t)sh.n, sh.device);
    launch_ivf_tile_i8(sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(), sh.tpass_off.get<int64_t>(), nlist, np,
                       d, sh.codes_i8.p, sh.xs8.get<float>(), st);
    sh.nflag.ensure(sizeof(int), sh.device);
    launch_ivf_i8_residual(sh.codes, sh.n, d, sh.nflag.get<unsigned>(), st);
    unsigned bits = 0;
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    float r2;
    std::memcpy(&r2, &bits, sizeof(r2));
    if (bits >= 0x7f800000u) {  // a non-finite row: the form does not apply (kFormSplit2Exact runs), as the fp16 image
        sh.i8_state = -1;
        sh.codes_i8.release();
        sh.xs8.release();
        return false;
    }
    sh.i8_rxmax = std::sqrt(r2) * 1.0001f;
    sh.i8_state = 1;
    return true;
}

// ‖x‖² of every stored row (L2 only): the decomposed scan form reads it with the codes
// (faiss-metal stores the same norms with its lists, MetalIndexIVFFlat.mm:313-318).
void compute_row_norms(IvfShard &sh, int d, int metric) {
    if (metric != kL2 || sh.n == 0) return;
    DeviceGuard g(sh.device);
    sh.xnorm.ensure(sizeof(float) * (size_t)sh.n, sh.device);
    launch_row_norms(sh.codes, sh.n, d, sh.xnorm.get<float>(), sh.stream);
    HIPANN_CHECK(hipStreamSynchronize(sh.stream));
}

}  // namespace

namespace hipann {

IvfIndex::~IvfIndex() {
    for (auto &s : shards) {
        s->quant.reset();
        DeviceGuard g(s->device);
        if (s->done) (void)hipEventDestroy(s->done);
        for (hipEvent_t e : s->app_ev)
            if (e) (void)hipEventDestroy(e);
        if (s->app_sync) (void)hipEventDestroy(s->app_sync);
        if (s->stream) (void)hipStreamDestroy(s->stream);
    }
}

// HIPANN_IVF_HOST_FALLBACK=1: the flagged queries of the exact forms are re-run from the host on the 3-term
// path after a readback of the flag count (the r01/r02 scheme; A/B only).  Default: on the device.
static bool host_fallback() {
    static const bool v = [] { const char *e = std::getenv("HIPANN_IVF_HOST_FALLBACK"); return e && std::atoi(e) != 0; }();
    return v;
}

// One shard: queries on the shard's device → D/I (nq × kout) on the same device, async on `st`.
// max‖x‖² of the shard (once): the rerank's error bound
float shard_xmax2(IvfShard &sh, int d, hipStream_t st) {
    if (sh.xmax2 >= 0.f) return sh.xmax2;
    const float *xn = sh.xnorm.get<float>();
    if (!xn) {
        sh.tmpnorm.ensure(sizeof(float) * (size_t)std::max<int64_t>(sh.n, 1), sh.device);
        launch_row_norms(sh.codes, sh.n, d, sh.tmpnorm.get<float>(), st);
        xn = sh.tmpnorm.get<float>();
    }
    sh.nflag.ensure(sizeof(int), sh.device);
    launch_ivf_max_norm(xn, sh.n, sh.nflag.get<unsigned>(), st);
    unsigned bits = 0;
    HIPANN_CHECK(hipMemcpyAsync(&bits, sh.nflag.p, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    sh.tmpnorm.release();
    float v;
    std::memcpy(&v, &bits, sizeof(v));
    sh.xmax2 = v;
    return v;
}

void ivf_shard_search(IvfIndex &ix, IvfShard &sh, int64_t nq, const float *xq, int k, int kout, float *D, int64_t *I,
                      hipStream_t st, int form_override, const int64_t *probes_in) {
    RoctxRange r_all("hipann.ivf.search_shard");
    DeviceGuard g(sh.device);
    const int nlist = ix.nlist, d = ix.d, metric = ix.metric;
    const int np = std::min(ix.nprobe, nlist);
    const float out_sign = metric == kIP ? -1.f : 1.f;
    // k > 64: per-slot direct scan + LDS sort (ivf_scan_slot_bigk), same plan / merge
    const bool bigk = k > 64;
    if (nq <= 0) return;
    // 1. coarse quantizer (FAISS: quantizer->search(n, x, nprobe) — Flat rules incl. nq < 20)
    sh.coarse_d.ensure((size_t)nq * np * sizeof(float), sh.device);
    sh.coarse_i.ensure((size_t)nq * np * sizeof(int64_t), sh.device);
    HIPANN_REQUIRE((int64_t)nq * np < (int64_t)0x7fffffff, "nq * nprobe too large");
    sh.slot_off.ensure(sizeof(int) * ((size_t)nq * np + 1), sh.device);
    // per-list counts and fill cursors, double-buffered by batch parity (ivf_planfill_q zeroes the other
    // parity's pair for the next batch; ivf_plan_q zeroes its own after use) — zeroed once per list count
    if (!sh.ccnt.p || !sh.cursor2.p || sh.plan_nlist != nlist) {
        sh.ccnt.ensure(sizeof(int) * 2 * kPlanCopies * (size_t)nlist, sh.device);
        sh.cursor2.ensure(sizeof(int) * 2 * kPlanCopies * (size_t)nlist, sh.device);
        HIPANN_CHECK(hipMemsetAsync(sh.ccnt.p, 0, sizeof(int) * 2 * kPlanCopies * (size_t)nlist, st));
        HIPANN_CHECK(hipMemsetAsync(sh.cursor2.p, 0, sizeof(int) * 2 * kPlanCopies * (size_t)nlist, st));
        sh.plan_nlist = nlist;
        sh.plan_batch = 0;
    }
    const int par = (int)(sh.plan_batch & 1u);
    const size_t pstride = (size_t)kPlanCopies * nlist;  // one parity's [copy][list] counts / cursors
    int *ccnt_cur = sh.ccnt.get<int>() + par * pstride, *ccnt_next = sh.ccnt.get<int>() + (1 - par) * pstride;
    int *cur_cur = sh.cursor2.get<int>() + par * pstride, *cur_next = sh.cursor2.get<int>() + (1 - par) * pstride;
    sh.qtot.ensure(sizeof(int) * (size_t)nq, sh.device);
    // this batch's counts must be zero on entry; the coarse select's count step adds to them, so if anything
    // throws before the plan has consumed them, zero them again on the way out
    struct CcntReset {
        int *p;
        int nlist;
        hipStream_t st;
        bool armed;
        ~CcntReset() {
            if (armed && std::uncaught_exceptions() > 0)
                (void)hipMemsetAsync(p, 0, sizeof(int) * kPlanCopies * (size_t)nlist, st);
        }
    } ccnt_reset{ccnt_cur, nlist, st, true};
    // the decomposed form needs float4 rows; other shapes take the direct kernel (also on the GPU)
    // the decomposed forms need float4 rows (else the direct kernel, also on the GPU); the MFMA kernel
    // keeps 16-lane lists (k <= 16) and the item's queries in LDS (else the VALU decomposed kernel)
    int req = form_override >= 0 ? form_override : ix.form;
    // request_k above kRerankMaxK on the exact forms (k + |tombstones|, faiss_index.cpp:713-715): the scans keep
    // their 16-lane lists but write every wave's list as a sub-list of the slot (mf_finish_item), and the rerank
    // takes the kf best candidates, certified against its kf-th merged key AND the smallest full sub-list's
    // 16th key (every pruned row lies above both).  Beyond kIvfSubMaxK: the 3-term scan.
    // kFormI8Exact always takes the sub-lists (its int8 filter needs the 64-deep rerank, ivf_mfma.hip)
    const bool sub_req = (((req == kFormHalfExact || req == kFormSplit2Exact) && kout > kRerankMaxK) ||
                          req == kFormI8Exact) && kout <= kIvfSubMaxK && !bigk;
    // kFormHalfExact: the fp16-image scan as the filter of the same rerank (else kFormSplit2Exact); kFormI8Exact: the
    // int8-image scan (else kFormSplit2Exact too)
    bool half = false, i8 = false;
    if (req == kFormHalfExact) {
        half = (kout <= kRerankMaxK || sub_req) && !bigk && ivf_mfma_h_supported(d, kRerankK) &&
               ensure_half_codes(sh, d, nlist, st);
        req = kFormSplit2Exact;
    } else if (req == kFormI8Exact) {
        i8 = sub_req && ivf_mfma_i8_supported(d, kRerankK) && ensure_i8_codes(sh, d, nlist, st);
        req = kFormSplit2Exact;
    }
    const bool img = half || i8;  // a tiled fp16 / int8 image and the one-term (or two-term) item scan
    // kFormSplit2Exact: the 2-term scan keeps kRerankK per list (per wave with sub-lists), the rerank makes the
    // results exact
    const bool want_exact = req == kFormSplit2Exact;
    if (want_exact) req = kout <= kRerankMaxK || sub_req ? kFormSplit2 : kFormSplit3;
    const int k_user = k;
    const int kscan = want_exact && req == kFormSplit2 ? kRerankK : k;
    int form = req != kFormDirect && !bigk && ivf_dot_supported(xq, d, sh.codes) ? req : kFormDirect;
    if (img) form = kFormSplit2;  // any d: the images are zero-padded to whole super-steps
    if (!img && ivf_form_split(form) && !ivf_mfma_bf_supported(xq, d, sh.codes, kscan, ivf_form_terms(form)))
        form = kFormDecomposed;
    if (form == kFormDecomposed && !ivf_mfma_supported(xq, d, sh.codes, kscan)) form = kFormDecomposedValu;
    const bool exact = want_exact && form == kFormSplit2;
    const bool sub = exact && sub_req;
    k = kscan;  // per-list k of the scan (the output keeps kout)
    // entries per (query, probe, chunk) slot, and the rerank's filter depth
    const int kslot = sub ? ivf_scan_sublists() * k : k;
    const int kfilt = sub ? (i8 ? 64 : std::min(64, std::max(kout + 4, 2 * kout))) : k;
    if (form_override < 0) {
        ix.last_form = exact ? (i8 ? kFormI8Exact : half ? kFormHalfExact : kFormSplit2Exact) : form;
        ix.last_kfilt = exact ? kfilt : 0;
        ix.last_sublists = sub ? ivf_scan_sublists() : 0;
    }
    const bool tiled = form == kFormDecomposed || ivf_form_split(form);  // the matrix-core scans
    const int group = i8 ? ivf_mfma_i8_group(d) : half ? ivf_mfma_h_group(d) : ivf_group_size(form, d);
    float xmax2 = 0.f;
    if (exact) {  // max‖x‖² (once per row set; nflag is its scratch, so before the plan resets the flag count)
        xmax2 = shard_xmax2(sh, d, st);
        sh.nflag.ensure(sizeof(int), sh.device);
        sh.flagged.ensure(sizeof(int) * (size_t)nq, sh.device);
    }
    unsigned *qbound = nullptr;
    if (tiled) {  // every query's bound starts at +inf (order-preserving bits 0xff800000), set by the plan
        sh.qbound.ensure(sizeof(unsigned) * (size_t)nq, sh.device);
        qbound = sh.qbound.get<unsigned>();
    }
    // the batch's query preparation, one launch before the coarse step (fp16 form): the fp16 query terms, 1/(t·s),
    // the split residuals and ‖q‖² (row_norms_f32's bits) for the coarse quantizer and the scan
    FlatShard &qsh0 = *sh.quant->shards[0];
    if (half) {
        sh.hsplit.ensure((size_t)ivf_half_qsplit_bytes(nq, d), sh.device);
        sh.hits.ensure(sizeof(float) * (size_t)nq, sh.device);
        sh.hres.ensure(sizeof(float) * 2 * (size_t)nq, sh.device);  // two- and one-term split residuals
        float *qn_out = nullptr;
        if (metric == kL2) {  // the quantizer's BLAS-form paths (nq >= 20) and the scan's L2 keys read ‖q‖²
            qsh0.qn.ensure(sizeof(float) * (size_t)nq, sh.device);
            qn_out = qsh0.qn.get<float>();
        }
        RoctxRange rr("hipann.ivf.prepare");
        launch_ivf_split_queries_h(xq, nq, d, sh.half_es, sh.hsplit.p, sh.hits.get<float>(), sh.hres.get<float>(), qn_out,
                                   st);
        qsh0.qn_given = qn_out ? xq : nullptr;
        qsh0.qn_given_nq = nq;
    } else if (i8) {
        // the int8 queries (units, scales, residuals) and ‖q‖² (row_norms_f32 itself: the coarse step's bits)
        sh.qi8.ensure((size_t)ivf_i8_qimg_bytes(nq, d), sh.device);
        sh.qs8.ensure(sizeof(float) * (size_t)nq, sh.device);
        sh.qres8.ensure(sizeof(float) * (size_t)nq, sh.device);
        float *qn_out = nullptr;
        if (metric == kL2) {
            qsh0.qn.ensure(sizeof(float) * (size_t)nq, sh.device);
            qn_out = qsh0.qn.get<float>();
            launch_row_norms(xq, nq, d, qn_out, st);
        }
        RoctxRange rr("hipann.ivf.prepare");
        launch_ivf_split_queries_i8(xq, nq, d, sh.qi8.p, sh.qs8.get<float>(), sh.qres8.get<float>(), st);
        qsh0.qn_given = qn_out ? xq : nullptr;
        qsh0.qn_given_nq = nq;
    }
    // the plan's per-query count step rides on the coarse probe select when that path is taken
    IvfPlanHook hook{sh.list_len.get<int>(), nlist, ivf_chunk_rows(), ccnt_cur, sh.slot_off.get<int>(),
                     sh.qtot.get<int>(), false};
    FlatShard &qsh = *sh.quant->shards[0];
    // HIPANN_IVF_SELECT_HOOK=0 (A/B): the count step in its own launch (ivf_count_q) instead of the select's tail
    static const bool hook_env = [] { const char *e = std::getenv("HIPANN_IVF_SELECT_HOOK"); return !e || std::atoi(e); }();
    if (probes_in) {
        // the probe lists come from the caller (the coarse step partitioned over ranks, hipann_ivf_coarse_device +
        // one all-gather): no quantizer launch; the plan counts the probes itself
        HIPANN_CHECK(hipMemcpyAsync(sh.coarse_i.p, probes_in, sizeof(int64_t) * (size_t)nq * np, hipMemcpyDeviceToDevice,
                                    st));
    } else {
        RoctxRange rr("hipann.ivf.coarse");
        qsh.plan_hook = ivf_plan_query_major() && hook_env ? &hook : nullptr;
        CoarseKeysScope ck(qsh);
        try {
            flat_shard_search(*sh.quant, qsh, nq, xq, np, np, sh.coarse_d.get<float>(), sh.coarse_i.get<int64_t>(), st);
        } catch (...) {
            qsh.plan_hook = nullptr;
            qsh.qn_given = nullptr;
            throw;
        }
    }
    qsh.plan_hook = nullptr;
    qsh.qn_given = nullptr;
    // 2. list-major work plan
    sh.cnt.ensure(sizeof(int) * (nlist + 1), sh.device);
    sh.bucket_off.ensure(sizeof(int) * (nlist + 1), sh.device);
    sh.item_off.ensure(sizeof(int) * (nlist + 1), sh.device);
    sh.bucket.ensure(sizeof(int) * (size_t)nq * np, sh.device);
    HIPANN_REQUIRE((int64_t)nq * np < (int64_t)0x7fffffff, "nq * nprobe too large");
    sh.slot_off.ensure(sizeof(int) * ((size_t)nq * np + 1), sh.device);
    {
    RoctxRange rr("hipann.ivf.plan");
    launch_ivf_plan(sh.coarse_i.get<int64_t>(), nq, np, sh.list_len.get<int>(), nlist, group, sh.cnt.get<int>(),
                    sh.bucket_off.get<int>(), sh.item_off.get<int>(), cur_cur, sh.bucket.get<int>(),
                    sh.slot_off.get<int>(), st, exact ? sh.nflag.get<int>() : nullptr, qbound, ccnt_cur,
                    sh.qtot.get<int>(), hook.done, ccnt_next, cur_next);
    }
    sh.plan_batch++;
    ccnt_reset.armed = false;
    // 3. scan: one k-list per (query, probe, row chunk) slot — every slot is written by exactly one item
    const size_t parts = (size_t)np * nq * sh.max_nch * kslot;
    HIPANN_REQUIRE((int64_t)np * nq * sh.max_nch < (int64_t)0x7fffffff, "too many partial lists");
    sh.part_d.ensure(parts * sizeof(float), sh.device);
    sh.part_i.ensure(parts * sizeof(int), sh.device);
    const int64_t max_items = ivf_max_items(nq, np, nlist, sh.max_nch, sh.n, group);
    const float *qn = nullptr;
    if (form != kFormDirect && metric == kL2) {
        const FlatShard &qs = *sh.quant->shards[0];
        if (probes_in && img) {
            qn = qsh0.qn.get<float>();  // the query preparation wrote ‖q‖² there (row_norms_f32's bits)
        } else if (!probes_in && qs.qn_of == xq && qs.qn_nq == nq) {
            // the coarse quantizer's ‖q‖² of the same queries, written by THIS call's coarse step (with probes_in
            // the quantizer did not run, and a cached pointer match may name a buffer whose contents changed)
            qn = qs.qn.get<float>();
        } else {
            sh.qn.ensure(sizeof(float) * (size_t)nq, sh.device);
            launch_row_norms(xq, nq, d, sh.qn.get<float>(), st);
            qn = sh.qn.get<float>();
        }
    }
    if (tiled && !img) ensure_tiled_codes(sh, d, nlist, st);
    if (img) {
        // query terms prepared before the coarse step
    } else if (ivf_form_split(form)) {
        sh.qsplit.ensure((size_t)ivf_mfma_bf_qsplit_bytes(nq, d, ivf_form_terms(form)), sh.device);
    }
    {
        RoctxRange rr("hipann.ivf.scan");
        ScopedTiming t(ix.timer_main, st);
        if (img) {
            // per 64-pass chunk key the latest item's round (HIPANN_IVF_FOLLOW=1 with a HIPANN_MH_FOLLOW=1 build, A/B
            // only: measured no better, ivf_mfma.hip); the
            // words carry the batch number, so a stale word is ignored and the buffer is zeroed only when allocated
            static const bool follow = [] { const char *e = std::getenv("HIPANN_IVF_FOLLOW"); return e && std::atoi(e); }();
            int nprog = 0;
            if (follow) {
                nprog = (int)std::min<int64_t>(1 << 20, (sh.h_off[nlist] / 32 + nlist) / 64 + 2);
                if (!sh.prog.p || sh.prog.bytes < sizeof(unsigned) * (size_t)nprog) {
                    sh.prog.ensure(sizeof(unsigned) * (size_t)nprog, sh.device);
                    HIPANN_CHECK(hipMemsetAsync(sh.prog.p, 0, sh.prog.bytes, st));
                }
            }
            // (int8: its query units, scales and residuals in the fp16 form's slots)
            launch_ivf_scan_mfma_h(xq, nq, i8 ? sh.qi8.p : sh.hsplit.p, i8 ? sh.qs8.get<float>() : sh.hits.get<float>(),
                                   i8 ? sh.qres8.get<float>() : sh.hres.get<float>(), sh.half_es, qn, d,
                                   metric, i8 ? sh.codes_i8.p : sh.codes_h.p, sh.tpass_off.get<int64_t>(), sh.xnorm.get<float>(),
                                   sh.list_off.get<int64_t>(), sh.list_len.get<int>(), sh.cnt.get<int>(), sh.bucket_off.get<int>(),
                                   sh.item_off.get<int>(), sh.bucket.get<int>(), sh.slot_off.get<int>(), nlist, np, k,
                                   max_items, qbound, sh.part_d.get<float>(), sh.part_i.get<int>(), st, true,
                                   sub ? 1 : 0, follow ? sh.prog.get<unsigned>() : nullptr, nprog,
                                   (unsigned)(sh.plan_batch + 1), i8 ? 1 : 0, i8 ? sh.xs8.get<float>() : nullptr);
        }
        else if (bigk)
            launch_ivf_scan_bigk(xq, d, metric, sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(),
                                 sh.coarse_i.get<int64_t>(),
                                 nq * np, np, sh.slot_off.get<int>(), nq * np * std::max(sh.max_nch, 1), k,
                                 sh.part_d.get<float>(), sh.part_i.get<int>(), st);
        else if (ivf_form_split(form))
            launch_ivf_scan_mfma_bf(ivf_form_terms(form), xq, nq, sh.qsplit.p, qn, d, metric, sh.codes_t.get<float>(),
                                    sh.tpass_off.get<int64_t>(), sh.xnorm.get<float>(), sh.list_off.get<int64_t>(),
                                    sh.list_len.get<int>(), sh.cnt.get<int>(), sh.bucket_off.get<int>(), sh.item_off.get<int>(),
                                    sh.bucket.get<int>(), sh.slot_off.get<int>(), nlist, np, k, max_items, qbound,
                                    sh.part_d.get<float>(), sh.part_i.get<int>(), st, sub ? 1 : 0);
        else if (form == kFormDecomposed)
            launch_ivf_scan_mfma(xq, qn, d, metric, sh.codes_t.get<float>(), sh.tpass_off.get<int64_t>(),
                                 sh.xnorm.get<float>(), sh.list_off.get<int64_t>(), sh.list_len.get<int>(),
                                 sh.cnt.get<int>(),
                                 sh.bucket_off.get<int>(), sh.item_off.get<int>(), sh.bucket.get<int>(),
                                 sh.slot_off.get<int>(), nlist, np, k, max_items, qbound, sh.part_d.get<float>(),
                                 sh.part_i.get<int>(), st);
        else
            launch_ivf_scan(xq, qn, d, metric, form, sh.codes, sh.xnorm.get<float>(), sh.list_off.get<int64_t>(),
                            sh.list_len.get<int>(), sh.cnt.get<int>(), sh.bucket_off.get<int>(), sh.item_off.get<int>(), sh.bucket.get<int>(),
                            sh.slot_off.get<int>(), nlist, np, nq, k, max_items, qbound, sh.part_d.get<float>(),
                            sh.part_i.get<int>(), st);
    }
    // 4. merge each query's partial lists (kFormSplit2Exact: merge + exact rerank + bound check)
    if (!exact) {
        ScopedTiming t(ix.timer_merge, st);
        launch_ivf_merge(sh.part_d.get<float>(), sh.part_i.get<int>(), sh.ids, sh.n, sh.slot_off.get<int>(), np, nq, k,
                         kout, out_sign, D, I, st);
        return;
    }
    // flagged queries re-run on the device in the direct form, each by the rerank wave that flagged it
    // (ivf_block_fallback inline: no host readback and no launch of its own); HIPANN_IVF_HOST_FALLBACK=1: from the
    // host on the 3-term path (A/B)
    const bool inline_fb = !host_fallback();
    int fb_cap = 0, fb_maxch = 1;
    if (inline_fb) {
        if (!sh.fb_total.p) {
            sh.fb_total.ensure(sizeof(unsigned long long), sh.device);
            HIPANN_CHECK(hipMemsetAsync(sh.fb_total.p, 0, sizeof(unsigned long long), st));
        }
        sh.fpd.ensure(sizeof(float) * (size_t)nq * np * kout, sh.device);
        sh.fpi.ensure(sizeof(long long) * (size_t)nq * np * kout, sh.device);
        // the parallel re-run of the batch's first fb_cap flagged queries (ivf_fallback_chunks): one wave per (query,
        // probe, chunk) item; its lists take ≤ 64 MB (fb_cap shrinks for long lists), later flagged queries re-run in
        // the flagging wave as before
        fb_maxch = sh.max_nch;
        const size_t per_f = (size_t)np * fb_maxch * kout * (sizeof(float) + sizeof(long long));
        fb_cap = (int)std::min<int64_t>({nq, 64, std::max<int64_t>(1, (int64_t)(((size_t)64 << 20) / per_f))});
        sh.fbc_d.ensure(sizeof(float) * (size_t)fb_cap * np * fb_maxch * kout, sh.device);
        sh.fbc_i.ensure(sizeof(long long) * (size_t)fb_cap * np * fb_maxch * kout, sh.device);
        if (sh.fbc_cap < fb_cap || !sh.fbc_done.p) {  // counters start (and are left) at zero
            sh.fbc_done.ensure(sizeof(unsigned) * (size_t)std::max(fb_cap, 64), sh.device);
            HIPANN_CHECK(hipMemsetAsync(sh.fbc_done.p, 0, sh.fbc_done.bytes, st));
            sh.fbc_cap = (int)(sh.fbc_done.bytes / sizeof(unsigned));
        }
    }
    {
        RoctxRange rr("hipann.ivf.rerank");
        ScopedTiming t(ix.timer_merge, st);
        launch_ivf_rerank(sh.part_d.get<float>(), sh.part_i.get<int>(), sh.slot_off.get<int>(), np, nq, kfilt, kout,
                          metric, xq, sh.codes, d, sh.ids, sh.n, 0, xmax2, D, I, sh.nflag.get<int>(),
                          sh.flagged.get<int>(), st, kSplit2Eps, i8 ? sh.i8_rxmax : half ? sh.half_rxmax : -1.f,
                          i8 ? sh.qres8.get<float>() : half ? sh.hres.get<float>() : nullptr, sh.coarse_i.get<int64_t>(),
                          sh.list_off.get<int64_t>(), nlist, qbound, img && metric == kL2 ? qn : nullptr, kslot,
                          sub ? 1 : 0, inline_fb ? sh.list_len.get<int>() : nullptr,
                          inline_fb ? sh.fpd.get<float>() : nullptr, inline_fb ? sh.fpi.get<long long>() : nullptr,
                          inline_fb ? sh.fb_total.get<unsigned long long>() : nullptr, fb_cap);
        if (fb_cap > 0)
            launch_ivf_fallback_chunks(sh.nflag.get<int>(), sh.flagged.get<int>(), fb_cap, np, fb_maxch, ivf_chunk_rows(),
                                       kout, metric, xq, sh.codes, d, sh.ids, 0, sh.coarse_i.get<int64_t>(),
                                       sh.list_off.get<int64_t>(), sh.list_len.get<int>(), nlist, sh.fbc_d.get<float>(),
                                       sh.fbc_i.get<long long>(), sh.fbc_done.get<unsigned>(), D, I,
                                       sh.fb_total.get<unsigned long long>(), st);
    }
    if (inline_fb) return;
    int nf = 0;
    HIPANN_CHECK(hipMemcpyAsync(&nf, sh.nflag.p, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPANN_CHECK(hipStreamSynchronize(st));
    if (nf <= 0) return;
    // flagged queries: re-run on the 3-term path (the batch's probe lists are kept for last_probes)
    ix.rerank_fallbacks += nf;
    const size_t pbytes = sizeof(int64_t) * (size_t)nq * np;
    sh.coarse_save.ensure(pbytes, sh.device);
    HIPANN_CHECK(hipMemcpyAsync(sh.coarse_save.p, sh.coarse_i.p, pbytes, hipMemcpyDeviceToDevice, st));
    sh.fq.ensure(sizeof(float) * (size_t)nf * d, sh.device);
    sh.fD.ensure(sizeof(float) * (size_t)nf * kout, sh.device);
    sh.fI.ensure(sizeof(int64_t) * (size_t)nf * kout, sh.device);
    launch_ivf_gather_queries(xq, sh.flagged.get<int>(), nf, d, sh.fq.get<float>(), st);
    {
        TimerPause p0(ix.timer_main), p1(ix.timer_merge);
        ivf_shard_search(ix, sh, nf, sh.fq.get<float>(), k_user, kout, sh.fD.get<float>(), sh.fI.get<int64_t>(), st,
                         kFormSplit3);
    }
    launch_ivf_scatter_results(sh.fD.get<float>(), sh.fI.get<int64_t>(), sh.flagged.get<int>(), nf, kout, D, I, st);
    HIPANN_CHECK(hipMemcpyAsync(sh.coarse_i.p, sh.coarse_save.p, pbytes, hipMemcpyDeviceToDevice, st));
}


// Grow a shard's CSR so that list l can take add[l] more rows: every list gets capacity max(cap, need + max(need / 4,
// 64)) rows — geometric growth (O(1) amortised copies per appended row, the doubling of MetalIndexFlat::add,
// MetalIndexFlat.mm:255-269, at ×1.25: a 10M × 768 table at ×2 would hold 61 GB of codes);
// borrowed storage is copied into owned buffers.  Live rows, labels, norms and the tiled images' passes move list by
// list (device-to-device, in order); the slack rows are zero (whole-table maxima read them).
static void ivf_relayout(IvfIndex &ix, IvfShard &sh, const std::vector<int64_t> &add) {
    const int nlist = ix.nlist, d = ix.d;
    hipStream_t st = sh.stream;
    // every list leaves with room for a quarter more than it will hold (≥ 64 rows): DuckDB's 2048-row chunks touch
    // most lists of a 1024-list index, so growing only the overflowing ones would relayout on nearly every append
    std::vector<int64_t> off(nlist + 1, 0);
    for (int l = 0; l < nlist; ++l) {
        const int64_t cap = sh.h_off[l + 1] - sh.h_off[l], need = sh.h_len[l] + add[l];
        const int64_t ncap = std::max(cap, need + std::max<int64_t>(need / 4, 64));
        off[l + 1] = off[l] + ncap;
    }
    const int64_t N = off[nlist];
    std::vector<int64_t> tp_old(nlist + 1, 0), tp(nlist + 1, 0);
    for (int l = 0; l < nlist; ++l) {
        tp_old[l + 1] = tp_old[l] + ceil_div(sh.h_off[l + 1] - sh.h_off[l], 32);
        tp[l + 1] = tp[l] + ceil_div(off[l + 1] - off[l], 32);
    }
    auto take = [](DevBuf &dst, DevBuf &src) {
        std::swap(dst.p, src.p);
        std::swap(dst.bytes, src.bytes);
        std::swap(dst.device, src.device);
    };
    // One array at a time — allocate its new layout, move its live lists (device-to-device, list by list, in order),
    // wait, swap, free the old one — so the transient peak is one array's old + new copy (2× the codes at most), not
    // every array twice.  `unit` = bytes per row (rows) or per 32-row pass (the tiled images); `pass` = per pass.
    auto move_array = [&](DevBuf &cur, const void *src_base, size_t unit, bool pass, size_t count) {
        auto nb = std::make_unique<DevBuf>();
        nb->ensure(unit * std::max<size_t>(count, 1), sh.device);
        HIPANN_CHECK(hipMemsetAsync(nb->p, 0, nb->bytes, st));
        for (int l = 0; l < nlist; ++l) {
            const int64_t len = sh.h_len[l];
            if (!len) continue;
            const int64_t o0 = pass ? tp_old[l] : sh.h_off[l], o1 = pass ? tp[l] : off[l];
            const int64_t cnt = pass ? ceil_div(len, 32) : len;  // passes holding live rows (past len: zero)
            HIPANN_CHECK(hipMemcpyAsync(static_cast<char *>(nb->p) + unit * (size_t)o1,
                                        static_cast<const char *>(src_base) + unit * (size_t)o0, unit * (size_t)cnt,
                                        hipMemcpyDeviceToDevice, st));
        }
        HIPANN_CHECK(hipStreamSynchronize(st));
        take(cur, *nb);  // nb now holds the old storage; freed here (borrowed storage: cur was empty)
    };
    move_array(sh.codes_buf, sh.codes, sizeof(float) * (size_t)d, false, (size_t)N);
    sh.codes = sh.codes_buf.get<float>();  // borrowed storage becomes owned here
    move_array(sh.ids_buf, sh.ids, sizeof(int64_t), false, (size_t)N);
    sh.ids = sh.ids_buf.get<int64_t>();
    sh.owns_codes = true;
    // L2 shards always leave with a norm array: a shard created empty (compute_row_norms skips n = 0) has none yet,
    // and ivf_append_rows writes the new rows' norms into it (the decomposed / fp16 scans read it)
    if (ix.metric == kL2) {
        if (sh.xnorm.p) {
            move_array(sh.xnorm, sh.xnorm.p, sizeof(float), false, (size_t)N);
        } else {
            sh.xnorm.ensure(sizeof(float) * (size_t)std::max<int64_t>(N, 1), sh.device);
            HIPANN_CHECK(hipMemsetAsync(sh.xnorm.p, 0, sh.xnorm.bytes, st));
        }
    }
    const bool img_h = sh.half_state > 0 && sh.codes_h.p, img_t = sh.codes_t.p != nullptr;
    if (img_h) move_array(sh.codes_h, sh.codes_h.p, (size_t)ivf_half_pass_bytes(d), true, (size_t)tp[nlist]);
    if (img_t)
        move_array(sh.codes_t, sh.codes_t.p, sizeof(float) * (size_t)ivf_mfma_pass_floats(d), true, (size_t)tp[nlist]);
    if (img_h || img_t) {
        sh.tpass_off.ensure(sizeof(int64_t) * (nlist + 1), sh.device);
        HIPANN_CHECK(hipMemcpyAsync(sh.tpass_off.p, tp.data(), sizeof(int64_t) * (nlist + 1), hipMemcpyHostToDevice, st));
        HIPANN_CHECK(hipStreamSynchronize(st));  // tp (host) is released on return
    } else {
        sh.tpass_off.release();  // recomputed from the new capacities when an image is built
    }
    upload_list_meta(sh, off, sh.h_len, nlist);
}

// IndexIVF::add_with_ids (FAISS 1.13.2, external): rows are assigned to their nearest centroid by the
// coarse quantizer (quantizer->assign, k = 1) and appended to their lists in insertion order; labels are `ids`
// or ntotal + i.  On the GPU copy this replaces the reference's invalidate-on-append (faiss_index.cpp:469): the new
// rows go into their lists' slack in HBM (ivf_relayout grows the lists that overflow, amortised), with their norms,
// the touched passes of the tiled images and running maxima — the cost of an append is the appended rows, not the
// table.
static void ivf_add_block(IvfIndex &ix, int64_t n, const float *xb, const int64_t *ids, int64_t base);

static void ivf_add_rows(IvfIndex &ix, int64_t n, const float *xb, const int64_t *ids) {
    // every shard's pending searches (possibly on other streams) finish before its buffers change
    std::vector<std::unique_ptr<FenceScope>> fences;
    for (auto &shp : ix.shards) fences.push_back(std::make_unique<FenceScope>(shp->fence, shp->stream, shp->device));
    // the int8 image (kFormI8Exact, opt-in) is not maintained in place: released, rebuilt at its next search
    for (auto &shp : ix.shards) {
        shp->i8_state = 0;
        shp->codes_i8.release();
        shp->xs8.release();
    }
    // FAISS assigns in blocks of 65536 rows (so the Flat nq < 20 direct-form rule applies per block); each block's
    // rows follow the previous block's in their lists (insertion order)
    const int64_t bs = 65536;
    for (int64_t r0 = 0; r0 < n; r0 += bs) {
        const int64_t m = std::min(bs, n - r0);
        ivf_add_block(ix, m, xb + r0 * (int64_t)ix.d, ids ? ids + r0 : nullptr, ix.ntotal());
    }
}

// One block of an add: rows to the device once; on shard 0's device the block's norms and, per shard, the block's
// maxima at that shard's fp16 scale (ivf_append_rows' statistics-only pass), then the coarse assignment on the GPU
// (shard 0's quantizer; every shard holds all centroids) — assignment and maxima come back in ONE readback, the block's
// only host wait.  The host folds the maxima (an image the new rows leave is dropped before it is re-tiled) and
// computes each row's physical destination; then per shard owning a list with new rows: grow the lists that overflow
// (ivf_relayout, amortised), one pinned upload (double-buffered: the next block writes the other buffer while this
// one's copy may still be queued), scatter each row straight into its list's slack (one kernel: codes, label, norm),
// re-tile the tiled images' touched passes.  Nothing waits for that tail: the next search is queued behind it.
static void ivf_add_block(IvfIndex &ix, int64_t n, const float *xb, const int64_t *ids, int64_t base) {
    RoctxRange r_all("hipann.ivf.add");
    const int d = ix.d, nlist = ix.nlist, metric = ix.metric;
    const int nsh = (int)ix.shards.size();
    IvfShard &s0 = *ix.shards[0];
    DeviceGuard g0(s0.device);
    hipStream_t st = s0.stream;
    // HIPANN_APPEND_PROF=1 (tuning): host-side phase times of each block on stderr
    static const bool prof = std::getenv("HIPANN_APPEND_PROF") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_0 = clk::now();
    auto us = [&](clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); };
    s0.app_rows.ensure(sizeof(float) * (size_t)n * d, s0.device);
    s0.app_norm.ensure(sizeof(float) * (size_t)n, s0.device);
    s0.app_assign.ensure(sizeof(int64_t) * (size_t)n, s0.device);
    HIPANN_CHECK(hipMemcpyAsync(s0.app_rows.p, xb, sizeof(float) * (size_t)n * d, hipMemcpyHostToDevice, st));
    double t_h2d = 0.0;
    if (prof) {
        HIPANN_CHECK(hipStreamSynchronize(st));
        t_h2d = us(t_0);
    }
    // the block's ‖x‖² (the table kernel's bits, the norms the append writes on shard 0) and per shard the maxima
    // [max ‖x‖², max |x|, max fp16 residual² at the shard's image scale]
    launch_row_norms(s0.app_rows.get<float>(), n, d, s0.app_norm.get<float>(), st);
    s0.app_stat.ensure(sizeof(unsigned) * 4 * (size_t)nsh, s0.device);
    unsigned *stat = s0.app_stat.get<unsigned>();
    for (int s = 0; s < nsh; ++s) {
        const IvfShard &sh = *ix.shards[s];
        const bool img_h = sh.half_state > 0 && sh.codes_h.p;
        launch_ivf_append_rows(s0.app_rows.get<float>(), s0.app_norm.get<float>(), nullptr, nullptr, n, d, nullptr,
                               nullptr, nullptr, nullptr, nullptr, 0, img_h ? std::ldexp(1.f, sh.half_es) : 0.f,
                               stat + 4 * s, st);
    }
    s0.app_cd.ensure(sizeof(float) * (size_t)n, s0.device);  // the assignment's distances (discarded)
    flat_shard_search(*s0.quant, *s0.quant->shards[0], n, s0.app_rows.get<float>(), 1, 1, s0.app_cd.get<float>(),
                      s0.app_assign.get<int64_t>(), st);
    s0.app_hassign.ensure(sizeof(int64_t) * (size_t)n + sizeof(unsigned) * 4 * (size_t)nsh);
    const int64_t *assign = s0.app_hassign.get<int64_t>();
    const unsigned *hstat = reinterpret_cast<const unsigned *>(assign + n);
    HIPANN_CHECK(hipMemcpyAsync(s0.app_hassign.p, s0.app_assign.p, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost,
                                st));
    HIPANN_CHECK(hipMemcpyAsync(const_cast<unsigned *>(hstat), stat, sizeof(unsigned) * 4 * (size_t)nsh,
                                hipMemcpyDeviceToHost, st));
    // the block's one host wait, polled (wait_event: no interrupt wake-up on the append's critical path)
    if (!s0.app_sync) HIPANN_CHECK(hipEventCreateWithFlags(&s0.app_sync, hipEventDisableTiming));
    HIPANN_CHECK(hipEventRecord(s0.app_sync, st));
    wait_event(s0.app_sync);
    const double t_assign = prof ? us(t_0) : 0.0;
    std::vector<int64_t> cnt(nlist, 0);
    for (int64_t i = 0; i < n; ++i) {
        HIPANN_REQUIRE(assign[i] >= 0 && assign[i] < nlist, "coarse assignment out of range");
        ++cnt[assign[i]];
    }
    for (int s = 0; s < nsh; ++s) {
        IvfShard &sh = *ix.shards[s];
        std::vector<int64_t> add(nlist, 0);
        int64_t add_s = 0;
        bool grow = !sh.owns_codes;
        for (int l = 0; l < nlist; ++l) {
            if (ix.owner[l] != s) continue;
            add[l] = cnt[l];
            add_s += add[l];
            if (sh.h_len[l] + add[l] > sh.h_off[l + 1] - sh.h_off[l]) grow = true;
        }
        if (!add_s) continue;
        // the block's maxima (over all its rows: for a shard that takes only some of them the bounds are at worst
        // slightly loose, never wrong) folded before anything is written
        const unsigned *hs = hstat + 4 * s;
        float v;
        std::memcpy(&v, &hs[0], sizeof(v));
        if (sh.xmax2 >= 0.f) sh.xmax2 = std::max(sh.xmax2, v);  // max ‖x‖² (the rerank bound's row term)
        if (sh.half_state > 0 && sh.codes_h.p) {
            float mx, r2;
            std::memcpy(&mx, &hs[1], sizeof(mx));
            std::memcpy(&r2, &hs[2], sizeof(r2));
            if (hs[1] >= 0x7f800000u) {  // a non-finite new entry: the fp16 form no longer applies (form 5 runs)
                sh.half_state = -1;
                sh.codes_h.release();
            } else if (mx >= std::ldexp(1.f, 14 - sh.half_es)) {  // outside the image's scale: rebuilt at the next search
                sh.half_state = 0;
                sh.codes_h.release();
            } else {
                sh.half_rxmax = std::max(sh.half_rxmax, std::sqrt(r2) * 1.0001f);
            }
        }
        DeviceGuard g(sh.device);
        hipStream_t ss = sh.stream;
        if (&sh != &s0) {  // the block's rows (and their norms) on this shard's device too
            sh.app_rows.ensure(sizeof(float) * (size_t)n * d, sh.device);
            sh.app_norm.ensure(sizeof(float) * (size_t)n, sh.device);
            HIPANN_CHECK(hipMemcpyAsync(sh.app_rows.p, xb, sizeof(float) * (size_t)n * d, hipMemcpyHostToDevice, ss));
            launch_row_norms(sh.app_rows.get<float>(), n, d, sh.app_norm.get<float>(), ss);
        }
        if (grow) ivf_relayout(ix, sh, add);
        // one pinned upload: [physical destination per row (−1: another shard's list) | label per row | the tiled
        // passes the rows touch | the new live length per list (int)]
        std::vector<int64_t> len = sh.h_len;
        std::vector<int64_t> tp0(nlist);
        int64_t np = 0, tp = 0;
        for (int l = 0; l < nlist; ++l) {
            tp0[l] = tp;
            tp += ceil_div(sh.h_off[l + 1] - sh.h_off[l], 32);
            if (add[l]) np += ceil_div(len[l] + add[l], 32) - len[l] / 32;
        }
        const size_t up_bytes = sizeof(int64_t) * (size_t)(2 * n + np) + sizeof(int) * (size_t)nlist;
        const int b = sh.app_buf;
        sh.app_buf ^= 1;
        if (sh.app_ev[b]) HIPANN_CHECK(hipEventSynchronize(sh.app_ev[b]));  // its copy two blocks ago (long done)
        HostBuf &hup = sh.app_hup[b];
        hup.ensure(up_bytes);
        int64_t *dst = hup.get<int64_t>(), *lab = dst + n, *passes = lab + n;
        int *newlen = reinterpret_cast<int *>(passes + np);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t l = assign[i];
            dst[i] = ix.owner[l] == s ? sh.h_off[l] + len[l]++ : -1;
            lab[i] = ids ? ids[i] : base + i;
        }
        int64_t pi = 0, maxlen = 0, live = 0;
        for (int l = 0; l < nlist; ++l) {
            for (int64_t p = sh.h_len[l] / 32; add[l] && p < ceil_div(len[l], 32); ++p) passes[pi++] = tp0[l] + p;
            HIPANN_REQUIRE(len[l] < (int64_t)0x7fffffff, "inverted list longer than 2^31-1 rows");
            newlen[l] = (int)len[l];
            maxlen = std::max(maxlen, len[l]);
            live += len[l];
        }
        sh.app_up.ensure(up_bytes, sh.device);
        HIPANN_CHECK(hipMemcpyAsync(sh.app_up.p, hup.p, up_bytes, hipMemcpyHostToDevice, ss));
        if (!sh.app_ev[b]) HIPANN_CHECK(hipEventCreateWithFlags(&sh.app_ev[b], hipEventDisableTiming));
        HIPANN_CHECK(hipEventRecord(sh.app_ev[b], ss));
        const int64_t *ddst = sh.app_up.get<int64_t>(), *dlab = ddst + n, *dpass = dlab + n;
        const int *dlen = reinterpret_cast<const int *>(dpass + np);
        const bool img_h = sh.half_state > 0 && sh.codes_h.p, img_t = sh.codes_t.p != nullptr;
        const float hscale = std::ldexp(1.f, sh.half_es);
        // one kernel: rows, labels and norms into their CSR rows, the new lengths
        launch_ivf_append_rows(sh.app_rows.get<float>(), sh.app_norm.get<float>(), ddst, dlab, n, d,
                               sh.codes_buf.get<float>(), sh.ids_buf.get<int64_t>(),
                               metric == kL2 ? sh.xnorm.get<float>() : nullptr, dlen, sh.list_len.get<int>(), nlist,
                               0.f, nullptr, ss);
        sh.h_len = len;
        sh.live = live;
        sh.max_nch = (int)std::max<int64_t>(1, ceil_div(maxlen, ivf_chunk_rows()));
        // the touched passes of the tiled images, re-tiled from the grown lists
        if (np > 0 && img_h)
            launch_ivf_tile_half(sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(), sh.tpass_off.get<int64_t>(),
                                 nlist, np, d, hscale, sh.codes_h.p, ss, dpass);
        if (np > 0 && img_t)
            launch_ivf_tile_codes(sh.codes, sh.list_off.get<int64_t>(), sh.list_len.get<int>(),
                                  sh.tpass_off.get<int64_t>(), nlist, np, d, sh.codes_t.get<float>(), ss, dpass);
        if (prof) {
            HIPANN_CHECK(hipStreamSynchronize(ss));
            std::fprintf(stderr, "hipann append: n %lld h2d %.0f us, assign %.0f us, shard %d done %.0f us (grow %d, %lld passes)\n",
                         (long long)n, t_h2d, t_assign, s, us(t_0), (int)grow, (long long)np);
        }
    }
}

}  // namespace hipann

extern "C" {

void *hipann_ivf_create(int d, int metric, int nlist, int nprobe, const float *centroids, const int64_t *list_offsets,
                        const int64_t *ids, const float *codes, const int *devices, int ndev, char *eb, int el) {
    return guard_ptr(eb, el, [&]() -> void * {
        int ndevs = 0;
        if (hipGetDeviceCount(&ndevs) != hipSuccess || ndevs <= 0) throw HipError("hipann: no HIP device");
        HIPANN_REQUIRE(d > 0 && nlist > 0, "d and nlist must be > 0");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 (L2) or 1 (IP)");
        HIPANN_REQUIRE(nprobe >= 1, "nprobe must be >= 1");
        HIPANN_REQUIRE(centroids && list_offsets, "null centroids / offsets");
        std::vector<int> devs;
        if (!devices || ndev <= 0) devs.push_back(0);
        else devs.assign(devices, devices + ndev);
        for (int dv : devs) HIPANN_REQUIRE(dv >= 0 && dv < ndevs, "invalid device id");
        const int64_t n = list_offsets[nlist];
        HIPANN_REQUIRE(list_offsets[0] == 0 && n >= 0, "list offsets must start at 0");
        for (int l = 0; l < nlist; ++l) HIPANN_REQUIRE(list_offsets[l + 1] >= list_offsets[l], "offsets not monotone");
        HIPANN_REQUIRE(n == 0 || (ids && codes), "null ids / codes");

        auto ix = std::make_unique<IvfIndex>();
        ix->d = d;
        ix->metric = metric;
        ix->nlist = nlist;
        ix->nprobe = nprobe;
        // size-balanced list → shard assignment (largest first onto the least-loaded shard)
        const int ns = (int)devs.size();
        std::vector<int> owner(nlist, 0);
        if (ns > 1) {
            std::vector<int> order(nlist);
            std::iota(order.begin(), order.end(), 0);
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                return list_offsets[a + 1] - list_offsets[a] > list_offsets[b + 1] - list_offsets[b];
            });
            std::vector<int64_t> load(ns, 0);
            for (int l : order) {
                const int s = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                owner[l] = s;
                load[s] += list_offsets[l + 1] - list_offsets[l];
            }
        }
        ix->owner = owner;
        for (int s = 0; s < ns; ++s) {
            auto sh = std::make_unique<IvfShard>();
            sh->device = devs[s];
            sh->stream = make_stream(devs[s]);
            DeviceGuard g(sh->device);
            std::vector<int64_t> off(nlist + 1, 0);
            for (int l = 0; l < nlist; ++l)
                off[l + 1] = off[l] + (owner[l] == s ? list_offsets[l + 1] - list_offsets[l] : 0);
            sh->n = off[nlist];
            sh->centroids_buf.ensure(sizeof(float) * (size_t)nlist * d, sh->device);
            HIPANN_CHECK(hipMemcpyAsync(sh->centroids_buf.p, centroids, sizeof(float) * (size_t)nlist * d,
                                        hipMemcpyHostToDevice, sh->stream));
            sh->centroids = sh->centroids_buf.get<float>();
            sh->codes_buf.ensure(sizeof(float) * (size_t)std::max<int64_t>(sh->n, 1) * d, sh->device);
            sh->ids_buf.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(sh->n, 1), sh->device);
            for (int l = 0; l < nlist; ++l) {
                if (owner[l] != s) continue;
                const int64_t cnt = list_offsets[l + 1] - list_offsets[l];
                if (!cnt) continue;
                HIPANN_CHECK(hipMemcpyAsync(sh->codes_buf.get<float>() + off[l] * d, codes + list_offsets[l] * d,
                                            sizeof(float) * (size_t)cnt * d, hipMemcpyHostToDevice, sh->stream));
                HIPANN_CHECK(hipMemcpyAsync(sh->ids_buf.get<int64_t>() + off[l], ids + list_offsets[l],
                                            sizeof(int64_t) * (size_t)cnt, hipMemcpyHostToDevice, sh->stream));
            }
            sh->codes = sh->codes_buf.get<float>();
            sh->ids = sh->ids_buf.get<int64_t>();
            sh->owns_codes = true;
            HIPANN_CHECK(hipStreamSynchronize(sh->stream));
            upload_list_meta(*sh, off, dense_lengths(off, nlist), nlist);
            compute_row_norms(*sh, d, metric);
            sh->quant = make_quantizer(d, metric, sh->centroids, nlist, sh->device, sh->stream);
            ix->shards.push_back(std::move(sh));
        }
        ix->peer = enable_peer_access(devs);
        return ix.release();
    });
}

void *hipann_ivf_create_device(int d, int metric, int nlist, int nprobe, const float *centroids_dev,
                               const int64_t *list_offsets, const int64_t *ids_dev, const float *codes_dev, int device,
                               int copy, char *eb, int el) {
    return guard_ptr(eb, el, [&]() -> void * {
        int ndevs = 0;
        if (hipGetDeviceCount(&ndevs) != hipSuccess || ndevs <= 0) throw HipError("hipann: no HIP device");
        HIPANN_REQUIRE(device >= 0 && device < ndevs, "invalid device");
        HIPANN_REQUIRE(d > 0 && nlist > 0 && nprobe >= 1, "bad arguments");
        HIPANN_REQUIRE(metric == kL2 || metric == kIP, "metric must be 0 (L2) or 1 (IP)");
        HIPANN_REQUIRE(centroids_dev && list_offsets, "null centroids / offsets");
        const int64_t n = list_offsets[nlist];
        HIPANN_REQUIRE(list_offsets[0] == 0 && n >= 0, "list offsets must start at 0");
        HIPANN_REQUIRE(n == 0 || (ids_dev && codes_dev), "null ids / codes");
        auto ix = std::make_unique<IvfIndex>();
        ix->d = d;
        ix->metric = metric;
        ix->nlist = nlist;
        ix->nprobe = nprobe;
        ix->owner.assign(nlist, 0);
        auto sh = std::make_unique<IvfShard>();
        sh->device = device;
        sh->stream = make_stream(device);
        sh->n = n;
        DeviceGuard g(device);
        HIPANN_CHECK(hipDeviceSynchronize());  // caller's writes to the inputs may still be in flight
        if (copy) {
            sh->centroids_buf.ensure(sizeof(float) * (size_t)nlist * d, device);
            sh->codes_buf.ensure(sizeof(float) * (size_t)std::max<int64_t>(n, 1) * d, device);
            sh->ids_buf.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(n, 1), device);
            HIPANN_CHECK(hipMemcpyAsync(sh->centroids_buf.p, centroids_dev, sizeof(float) * (size_t)nlist * d,
                                        hipMemcpyDeviceToDevice, sh->stream));
            if (n) {
                HIPANN_CHECK(hipMemcpyAsync(sh->codes_buf.p, codes_dev, sizeof(float) * (size_t)n * d,
                                            hipMemcpyDeviceToDevice, sh->stream));
                HIPANN_CHECK(hipMemcpyAsync(sh->ids_buf.p, ids_dev, sizeof(int64_t) * (size_t)n,
                                            hipMemcpyDeviceToDevice, sh->stream));
            }
            sh->centroids = sh->centroids_buf.get<float>();
            sh->codes = sh->codes_buf.get<float>();
            sh->ids = sh->ids_buf.get<int64_t>();
            sh->owns_codes = true;
        } else {
            sh->centroids = centroids_dev;
            sh->codes = codes_dev;
            sh->ids = ids_dev;
        }
        std::vector<int64_t> off(list_offsets, list_offsets + nlist + 1);
        upload_list_meta(*sh, off, dense_lengths(off, nlist), nlist);
        compute_row_norms(*sh, d, metric);
        sh->quant = make_quantizer(d, metric, sh->centroids, nlist, device, sh->stream);
        ix->shards.push_back(std::move(sh));
        return ix.release();
    });
}

static int ivf_search_host(IvfIndex &ix, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I) {
    HIPANN_REQUIRE(k > 0, "k must be > 0");
    HIPANN_REQUIRE(k <= HIPANN_MAX_K, "k larger than HIPANN_MAX_K");
    HIPANN_REQUIRE(nq >= 0 && (nq == 0 || (xq && D && I)), "invalid arguments");
    const float pad = ix.metric == kIP ? -__builtin_inff() : __builtin_inff();
    const int64_t ntot = ix.ntotal();
    ix.last_nq = nq;
    ix.last_np = std::min(ix.nprobe, ix.nlist);
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
    for (auto &shp : ix.shards) {
        IvfShard &sh = *shp;
        DeviceGuard g(sh.device);
        sh.q.ensure(qbytes, sh.device);
        sh.out_d.ensure(ob * sizeof(float), sh.device);
        sh.out_i.ensure(ob * sizeof(int64_t), sh.device);
        FenceScope fs(sh.fence, sh.stream, sh.device);
        if (qbytes <= kKernelCopyMax) launch_copy_words(host_device_ptr(ix.h_q.p), sh.q.p, qbytes, sh.stream);
        else HIPANN_CHECK(hipMemcpyAsync(sh.q.p, ix.h_q.p, qbytes, hipMemcpyHostToDevice, sh.stream));
        ivf_shard_search(ix, sh, nq, sh.q.get<float>(), keff, kout, sh.out_d.get<float>(), sh.out_i.get<int64_t>(),
                         sh.stream);
        if (ix.shards.size() > 1) {  // shard 0's stream waits for it on the device (no host wait per shard)
            if (!sh.done) HIPANN_CHECK(hipEventCreateWithFlags(&sh.done, hipEventDisableTiming));
            HIPANN_CHECK(hipEventRecord(sh.done, sh.stream));
        }
    }
    ix.h_d.ensure(ob * sizeof(float));
    ix.h_i.ensure(ob * sizeof(int64_t));
    IvfShard &s0 = *ix.shards[0];
    if (ix.shards.size() == 1) {
        DeviceGuard g(s0.device);
        if (ob * sizeof(int64_t) <= kKernelCopyMax) {
            launch_copy_words(s0.out_d.p, host_device_ptr(ix.h_d.p), ob * sizeof(float), s0.stream);
            launch_copy_words(s0.out_i.p, host_device_ptr(ix.h_i.p), ob * sizeof(int64_t), s0.stream);
        } else {
            HIPANN_CHECK(hipMemcpyAsync(ix.h_d.p, s0.out_d.p, ob * sizeof(float), hipMemcpyDeviceToHost, s0.stream));
            HIPANN_CHECK(hipMemcpyAsync(ix.h_i.p, s0.out_i.p, ob * sizeof(int64_t), hipMemcpyDeviceToHost, s0.stream));
        }
        HIPANN_CHECK(hipStreamSynchronize(s0.stream));
    } else {
        const int np = (int)ix.shards.size();
        ix.gather_d.ensure(ob * np * sizeof(float), s0.device);
        ix.gather_i.ensure(ob * np * sizeof(int64_t), s0.device);
        ix.merged_d.ensure(ob * sizeof(float), s0.device);
        ix.merged_i.ensure(ob * sizeof(int64_t), s0.device);
        DeviceGuard g0(s0.device);
        for (int p = 0; p < np; ++p) {
            IvfShard &sh = *ix.shards[p];
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
        HIPANN_CHECK(hipStreamSynchronize(s0.stream));
    }
    std::memcpy(D, ix.h_d.p, ob * sizeof(float));
    std::memcpy(I, ix.h_i.p, ob * sizeof(int64_t));
    return 0;
}

int hipann_ivf_search(void *h, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        return ivf_search_host(*vx, nq, xq, k, D, I);
    });
}

int hipann_ivf_search_np(void *h, int nprobe, int64_t nq, const float *xq, int64_t k, float *D, int64_t *I, char *eb,
                         int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        if (nprobe <= 0) return ivf_search_host(*vx, nq, xq, k, D, I);
        // the call's nprobe, read and restored under the handle's lock (concurrent connections with
        // different SearchParametersIVF never see each other's value)
        const int saved = vx->nprobe;
        vx->nprobe = nprobe;
        try {
            const int rc = ivf_search_host(*vx, nq, xq, k, D, I);
            vx->nprobe = saved;
            return rc;
        } catch (...) {
            vx->nprobe = saved;
            throw;
        }
    });
}

int hipann_ivf_search_device(void *h, int64_t nq, const float *xq_dev, int64_t k, float *D_dev, int64_t *I_dev,
                             void *stream, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        HIPANN_REQUIRE(vx->shards.size() == 1, "device search needs a single-device index");
        HIPANN_REQUIRE(k > 0 && k <= HIPANN_MAX_K, "k out of range");
        IvfShard &sh = *vx->shards[0];
        hipStream_t st = static_cast<hipStream_t>(stream);  // NULL = the default (null) stream
        vx->last_nq = nq;
        vx->last_np = std::min(vx->nprobe, vx->nlist);
        const int keff = (int)std::min<int64_t>(k, std::max<int64_t>(sh.live, 1));
        FenceScope fs(sh.fence, st, sh.device);  // the previous call's kernels may still use this shard's scratch
        ivf_shard_search(*vx, sh, nq, xq_dev, keff, (int)k, D_dev, I_dev, st);
        return 0;
    });
}

int hipann_ivf_coarse_device(void *h, int64_t nq, const float *xq_dev, int64_t *probes_dev, void *stream, char *eb,
                             int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        HIPANN_REQUIRE(vx->shards.size() == 1, "device coarse step needs a single-device index");
        HIPANN_REQUIRE(nq >= 0 && (nq == 0 || (xq_dev && probes_dev)), "invalid arguments");
        if (nq == 0) return 0;
        IvfShard &sh = *vx->shards[0];
        DeviceGuard g(sh.device);
        hipStream_t st = static_cast<hipStream_t>(stream);
        const int np = std::min(vx->nprobe, vx->nlist);
        FenceScope fs(sh.fence, st, sh.device);
        sh.app_cd.ensure(sizeof(float) * (size_t)nq * np, sh.device);
        // FAISS quantizer->search(nq, x, nprobe): the Flat rules of the coarse quantizer (exact fp32 products)
        CoarseKeysScope ck(*sh.quant->shards[0]);
        flat_shard_search(*sh.quant, *sh.quant->shards[0], nq, xq_dev, np, np, sh.app_cd.get<float>(), probes_dev, st);
        return 0;
    });
}

int hipann_ivf_search_probes_device(void *h, int64_t nq, const float *xq_dev, const int64_t *probes_dev, int64_t k,
                                    float *D_dev, int64_t *I_dev, void *stream, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        HIPANN_REQUIRE(vx->shards.size() == 1, "device search needs a single-device index");
        HIPANN_REQUIRE(k > 0 && k <= HIPANN_MAX_K, "k out of range");
        HIPANN_REQUIRE(nq >= 0 && (nq == 0 || (xq_dev && probes_dev && D_dev && I_dev)), "invalid arguments");
        IvfShard &sh = *vx->shards[0];
        hipStream_t st = static_cast<hipStream_t>(stream);
        vx->last_nq = nq;
        vx->last_np = std::min(vx->nprobe, vx->nlist);
        const int keff = (int)std::min<int64_t>(k, std::max<int64_t>(sh.live, 1));
        FenceScope fs(sh.fence, st, sh.device);
        ivf_shard_search(*vx, sh, nq, xq_dev, keff, (int)k, D_dev, I_dev, st, -1, probes_dev);
        return 0;
    });
}

int hipann_ivf_add(void *h, int64_t n, const float *xb, const int64_t *ids, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        HIPANN_REQUIRE(n >= 0 && (n == 0 || xb), "invalid vectors");
        if (n > 0) ivf_add_rows(*vx, n, xb, ids);
        return 0;
    });
}

int hipann_ivf_nlist(void *h) {
    if (!h || static_cast<IndexBase *>(h)->kind != Kind::IVF) return -1;
    return static_cast<IvfIndex *>(h)->nlist;
}

int hipann_ivf_get_nprobe(void *h) {
    if (!h || static_cast<IndexBase *>(h)->kind != Kind::IVF) return -1;
    auto *vx = static_cast<IvfIndex *>(h);
    std::lock_guard<std::mutex> lk(vx->mu);
    return vx->nprobe;
}

int hipann_ivf_export(void *h, float *centroids, int64_t *list_offsets, int64_t *ids, float *codes, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h, "null index");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        const int nlist = vx->nlist, d = vx->d;
        std::vector<int64_t> off(nlist + 1, 0);
        for (int l = 0; l < nlist; ++l) {
            const IvfShard &sh = *vx->shards[vx->owner[l]];
            off[l + 1] = off[l] + sh.h_len[l];  // live rows (the shard's physical list may hold append slack)
        }
        if (list_offsets) std::memcpy(list_offsets, off.data(), sizeof(int64_t) * (nlist + 1));
        IvfShard &s0 = *vx->shards[0];
        if (centroids) {
            DeviceGuard g(s0.device);
            HIPANN_CHECK(hipMemcpyAsync(centroids, s0.centroids, sizeof(float) * (size_t)nlist * d, hipMemcpyDeviceToHost,
                                        s0.stream));
            HIPANN_CHECK(hipStreamSynchronize(s0.stream));
        }
        for (int l = 0; l < nlist && (ids || codes); ++l) {
            IvfShard &sh = *vx->shards[vx->owner[l]];
            const int64_t len = off[l + 1] - off[l];
            if (!len) continue;
            DeviceGuard g(sh.device);
            if (codes)
                HIPANN_CHECK(hipMemcpyAsync(codes + off[l] * d, sh.codes + sh.h_off[l] * d, sizeof(float) * (size_t)len * d,
                                            hipMemcpyDeviceToHost, sh.stream));
            if (ids)
                HIPANN_CHECK(hipMemcpyAsync(ids + off[l], sh.ids + sh.h_off[l], sizeof(int64_t) * (size_t)len,
                                            hipMemcpyDeviceToHost, sh.stream));
        }
        for (auto &shp : vx->shards) {
            DeviceGuard g(shp->device);
            HIPANN_CHECK(hipStreamSynchronize(shp->stream));
        }
        return 0;
    });
}

int hipann_ivf_last_probes(void *h, int64_t *probes, int64_t cap, char *eb, int el) {
    return guard_int(eb, el, [&]() -> int {
        HIPANN_REQUIRE(h && probes, "null argument");
        auto *ix = static_cast<IndexBase *>(h);
        HIPANN_REQUIRE(ix->kind == Kind::IVF, "not an IVFFlat index");
        auto *vx = static_cast<IvfIndex *>(ix);
        std::lock_guard<std::mutex> lk(vx->mu);
        const int64_t m = vx->last_nq * vx->last_np;
        HIPANN_REQUIRE(cap >= m, "probe buffer too small");
        if (m == 0) return 0;
        IvfShard &sh = *vx->shards[0];
        DeviceGuard g(sh.device);
        HIPANN_CHECK(hipStreamSynchronize(sh.stream));
        HIPANN_CHECK(hipDeviceSynchronize());
        HIPANN_CHECK(hipMemcpy(probes, sh.coarse_i.p, sizeof(int64_t) * (size_t)m, hipMemcpyDeviceToHost));
        return 0;
    });
}

int hipann_ivf_set_nprobe(void *h, int nprobe) {
    if (!h || nprobe < 1) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::IVF) return -1;
    auto *vx = static_cast<IvfIndex *>(ix);
    std::lock_guard<std::mutex> lk(vx->mu);
    vx->nprobe = nprobe;
    return 0;
}

int hipann_ivf_set_form(void *h, int form) {
    if (!h || form < kFormDecomposed || form > kFormI8Exact) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::IVF) return -1;
    auto *vx = static_cast<IvfIndex *>(ix);
    std::lock_guard<std::mutex> lk(vx->mu);
    vx->form = form;
    return 0;
}

int64_t hipann_ivf_rerank_fallbacks(void *h) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::IVF) return -1;
    auto *vx = static_cast<IvfIndex *>(ix);
    std::lock_guard<std::mutex> lk(vx->mu);
    int64_t t = vx->rerank_fallbacks;  // host re-runs (HIPANN_IVF_HOST_FALLBACK)
    for (auto &sh : vx->shards) {       // + the device re-runs' running count
        if (!sh->fb_total.p) continue;
        DeviceGuard g(sh->device);
        unsigned long long v = 0;
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        if (hipMemcpy(&v, sh->fb_total.p, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        t += (int64_t)v;
    }
    return t;
}

int hipann_ivf_get_form(void *h) {
    if (!h) return -1;
    auto *ix = static_cast<IndexBase *>(h);
    if (ix->kind != Kind::IVF) return -1;
    return static_cast<IvfIndex *>(ix)->form;
}

}  // extern "C"
