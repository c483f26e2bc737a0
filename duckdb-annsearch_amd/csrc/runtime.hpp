// runtime.hpp — device buffers, per-handle streams/scratch and the index objects behind hip_ann.h.
#pragma once
#include "common.hpp"
#include <cstdlib>
#include <ctime>
#include <memory>
#include <mutex>
#include <vector>

namespace hipann {

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev) {
        HIPANN_CHECK(hipGetDevice(&prev));
        if (prev != dev) HIPANN_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// Device allocation that grows on demand (never shrinks) — the per-handle scratch arena.
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int device = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) { DeviceGuard g(device); (void)hipFree(p); }
        p = nullptr;
        bytes = 0;
    }
    template <typename T> T *get() const { return static_cast<T *>(p); }
    // Grow to at least `need` bytes on `dev`.  Contents are NOT preserved.  A buffer that grows again (per-batch
    // scratch whose size follows the longest list as appends lengthen it) takes a quarter of headroom below 1 GiB, so
    // a run of appends does not free and re-allocate it — each hipFree synchronises the device — on every search
    // (HIPANN_BUF_HEADROOM=0: exact sizes, A/B).
    void ensure(size_t need, int dev) {
        if (need <= bytes && dev == device && p) return;
        static const bool headroom = [] { const char *e = std::getenv("HIPANN_BUF_HEADROOM"); return !e || std::atoi(e); }();
        const bool regrow = p && dev == device && headroom && need < ((size_t)1 << 30);
        release();
        device = dev;
        DeviceGuard g(dev);
        size_t alloc = need < 256 ? 256 : need;
        if (regrow) alloc += alloc / 4;
        HIPANN_CHECK(hipMalloc(&p, alloc));
        bytes = alloc;
    }
};

// Pinned host staging buffer.
struct HostBuf {
    void *p = nullptr;
    size_t bytes = 0;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    ~HostBuf() { if (p) (void)hipHostFree(p); }
    // (returns true when it allocated: the contents are undefined then)
    bool ensure(size_t need, unsigned flags = hipHostMallocDefault) {
        if (need <= bytes && p) return false;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        HIPANN_CHECK(hipHostMalloc(&p, need < 256 ? 256 : need, flags));
        bytes = need < 256 ? 256 : need;
        return true;
    }
    template <typename T> T *get() const { return static_cast<T *>(p); }
};

// HIP-event timing of a kernel across calls (bench.py reads the average).
struct KernelTimer {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
    int device = 0;
    ~KernelTimer() { clear(); }
    void clear() {
        for (auto &e : ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
        ev.clear();
        used = 0;
    }
    void reset(bool enable, int dev) { clear(); on = enable; device = dev; }
    // Returns the event pair to record around a launch (nullptr pair when off).
    std::pair<hipEvent_t, hipEvent_t> next() {
        if (!on) return {nullptr, nullptr};
        if (used == ev.size()) {
            hipEvent_t a, b;
            // timing-only events: no system-scope fence (an L2 writeback + invalidate per record, ≈5 µs of
            // idle GPU between the timed kernel and the next launch); average_ms reads them after a sync
            HIPANN_CHECK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
            HIPANN_CHECK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
            ev.push_back({a, b});
        }
        return ev[used++];
    }
    double average_ms() {
        if (!used) return 0.0;
        double tot = 0.0;
        for (size_t i = 0; i < used; ++i) {
            HIPANN_CHECK(hipEventSynchronize(ev[i].second));
            float ms = 0.f;
            HIPANN_CHECK(hipEventElapsedTime(&ms, ev[i].first, ev[i].second));
            tot += ms;
        }
        return tot / (double)used;
    }
};

struct ScopedTiming {
    hipEvent_t b;
    hipStream_t s;
    ScopedTiming(KernelTimer &t, hipStream_t st) : s(st) {
        auto e = t.next();
        b = e.second;
        if (e.first) HIPANN_CHECK(hipEventRecord(e.first, st));
    }
    ~ScopedTiming() { if (b) (void)hipEventRecord(b, s); }
};

// roctx ranges around the host stages of a call (HIPANN_ROCTX=1; off by default, then a scope costs one branch):
// `rocprofv3 --marker-trace` shows each stage's enqueue span beside the kernels it launched (profiles/r06/).
bool roctx_enabled();
void roctx_push(const char *name);
void roctx_pop();
struct RoctxRange {
    bool on;
    explicit RoctxRange(const char *name) : on(roctx_enabled()) { if (on) roctx_push(name); }
    ~RoctxRange() { if (on) roctx_pop(); }
    RoctxRange(const RoctxRange &) = delete;
    RoctxRange &operator=(const RoctxRange &) = delete;
};

// Pauses a timer for a scope (the exact forms' re-runs of flagged queries stay out of the main kernel's
// timing, which the roofline reads).
struct TimerPause {
    KernelTimer &t;
    bool was;
    explicit TimerPause(KernelTimer &tt) : t(tt), was(tt.on) { t.on = false; }
    ~TimerPause() { t.on = was; }
};

// Orders a handle's calls across streams.  Every search / add of a shard runs its kernels on the caller's
// stream (device API) or the shard's own (host API) and reuses the shard's scratch (plan counts, partial
// lists, flags).  The handle mutex only covers enqueueing, so a call on another stream must not start
// before the previous call's kernels are done with that scratch: each call waits for the event the
// previous call recorded (when the streams differ) and records its own at the end.
// Host waits by polling instead of blocking.  hipStreamSynchronize / hipEventSynchronize may put the thread to
// sleep until the completion interrupt, whose wake-up adds tens of µs to every short call (r05 C2 traces: a 44 µs
// idle gap before each search after the previous one's synchronisation).  HIPANN_SPIN_WAIT=0 (A/B): the blocking
// calls.
inline bool spin_wait() {
    static const bool v = [] { const char *e = std::getenv("HIPANN_SPIN_WAIT"); return !e || std::atoi(e) != 0; }();
    return v;
}
// The spin is bounded: after HIPANN_SPIN_US microseconds (default 2000 — the C2 batch and every IVF batch finish
// inside it; a 10M-row Flat batch of ≈8 ms pays one wake-up, < 1 %) the wait blocks, so a long search does not hold a
// host core (DuckDB's worker pool runs concurrent searches).
inline int64_t spin_budget_ns() {
    static const int64_t v = [] {
        const char *e = std::getenv("HIPANN_SPIN_US");
        return (int64_t)(e ? std::atoll(e) : 2000) * 1000;
    }();
    return v;
}
inline int64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}
// until `ev` has completed (hipEventQuery in a pause loop; errors surface as from the blocking call)
inline void wait_event(hipEvent_t ev) {
    if (spin_wait()) {
        const int64_t t_end = mono_ns() + spin_budget_ns();
        for (unsigned it = 1;; ++it) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) HIPANN_CHECK(e);
            for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
            if ((it & 63) == 0 && mono_ns() > t_end) break;
        }
    }
    HIPANN_CHECK(hipEventSynchronize(ev));
}
// until the token word `tok` (written by launch_post_words, the last work on `st`) reads `token`: every earlier
// kernel on the stream has completed then.  The stream is queried now and then, so a failed or finished stream
// ends the wait too (its error raised as hipStreamSynchronize would).
inline void wait_posted(const volatile unsigned *tok, unsigned token, hipStream_t st) {
    if (spin_wait()) {
        const int64_t t_end = mono_ns() + spin_budget_ns();
        for (unsigned it = 1;; ++it) {
            if (__atomic_load_n(tok, __ATOMIC_ACQUIRE) == token) return;
            if ((it & 1023) == 0) {
                const hipError_t e = hipStreamQuery(st);
                if (e == hipSuccess) return;
                if (e != hipErrorNotReady) HIPANN_CHECK(hipStreamSynchronize(st));
                if (mono_ns() > t_end) break;
            }
            __builtin_ia32_pause();
        }
    }
    HIPANN_CHECK(hipStreamSynchronize(st));
}

struct StreamFence {
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool armed = false;
    bool multi = false;  // a call has arrived on a different stream than its predecessor: events from now on
    bool ev_valid = false;  // ev holds the previous call's end
    int device = 0;
    StreamFence() = default;
    StreamFence(const StreamFence &) = delete;
    StreamFence &operator=(const StreamFence &) = delete;
    ~StreamFence() { if (ev) { DeviceGuard g(device); (void)hipEventDestroy(ev); } }
    // Adaptive.  While every call of the handle comes on one stream nothing is recorded per call — an event record is
    // a marker packet the next kernel waits behind (≈6 µs of idle GPU between consecutive searches on one stream, r05
    // kernel traces).  The first call on a different stream synchronises the handle's device once (no event of the
    // previous call exists; its stream may have been destroyed since) and switches the fence to events: from then on
    // every call records one at its end, and a call on another stream waits for it on the device (hipStreamWaitEvent)
    // — per-connection streams cost one marker per call, not a device-wide drain per alternation.
    // HIPANN_FENCE_EAGER=1: events from the first call.
    static bool eager() {
        static const bool v = [] { const char *e = std::getenv("HIPANN_FENCE_EAGER"); return e && std::atoi(e) != 0; }();
        return v;
    }
    void enter(hipStream_t st) {
        if (!armed || st == last) return;
        if (ev_valid) {
            HIPANN_CHECK(hipStreamWaitEvent(st, ev, 0));
        } else {
            DeviceGuard g(device);
            HIPANN_CHECK(hipDeviceSynchronize());
        }
        multi = true;
    }
    void leave(hipStream_t st, int dev) {
        if (eager() || multi) {
            if (!ev) {
                DeviceGuard g(dev);
                HIPANN_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            }
            HIPANN_CHECK(hipEventRecord(ev, st));
            ev_valid = true;
        }
        device = dev;
        last = st;
        armed = true;
    }
};
struct FenceScope {
    StreamFence &f;
    hipStream_t st;
    int dev;
    FenceScope(StreamFence &ff, hipStream_t s, int d) : f(ff), st(s), dev(d) { f.enter(st); }
    ~FenceScope() {
        try { f.leave(st, dev); } catch (...) {}
    }
};

enum class Kind { Flat = 1, IVF = 2 };

// One contiguous row range of a Flat index resident on one device.
struct FlatShard {
    int device = 0;
    int64_t n = 0, cap = 0;
    int64_t label_offset = 0;
    float *xb = nullptr;  // n × d fp32 (owned unless borrowed)
    bool owns = true;
    DevBuf xb_buf;        // owned storage
    DevBuf xn;            // ‖x‖² (L2 only)
    hipStream_t stream = nullptr;
    // scratch
    DevBuf q, qn, part_d, part_i, out_d, out_i;
    // IVF coarse quantizer only: the plan's per-query count step fused into the probe select (set by
    // ivf_shard_search around its coarse call; done = the select consumed it)
    struct IvfPlanHook *plan_hook = nullptr;
    const float *qn_of = nullptr;  // sh.qn holds ‖q‖² of these queries (the last search's, nq of them)
    int64_t qn_nq = 0;
    // set by the caller before a search: sh.qn already holds ‖q‖² of these queries (the IVF query preparation
    // computed it), so the search does not launch row_norms again
    const float *qn_given = nullptr;
    int64_t qn_given_nq = 0;
    DevBuf keys, run_d, run_i, run2_d, run2_i;  // k > 64 path
    DevBuf mid_d, mid_i;                        // two-level merge of the direct scan's per-wave lists
    DevBuf qsplit;                              // split-bf16 form: the batch's queries as bf16 terms
    // kFlatSplit2Exact: max row ‖x‖² (the rerank's error bound; −1 until computed / after an add), the
    // flagged queries of the last batch and the re-run's buffers
    float xmax2 = -1.f;
    DevBuf nflag, flagged, fq, fD, fI, tmpnorm;
    DevBuf crd, cri, covf, nflag2, flagged2;  // form 4: flagged queries reranked over all their buffered candidates
    // kFlatBf16Exact: tiled bf16 image of the rows (built at the first search after an add) and the
    // batch's query image
    DevBuf xb16, qimg, seed;
    DevBuf cand;  // bounded passes: per-(query, split) candidate buffers and counts
    bool xb16_ok = false;
    bool keys_bf3 = false;    // the small-table key GEMM on the bf16 matrix cores (3 terms): the IVF coarse step
    float bf16_rxmax = 0.f;  // max over rows of ‖bf16(x) − x‖ (the rerank's bound)
    // kFlatI8Exact: tiled int8 image, per-row scales, max row residual ‖x − s·x̂‖; the batch's query scales and
    // residuals (the rerank's query term)
    DevBuf xi8, xscale, qscale, qres;
    bool xi8_ok = false;
    float i8_rxmax = 0.f;
    StreamFence fence;       // cross-stream ordering of this shard's calls
    HostBuf h_nflag;         // the launch phase's flag count, read back with the results (flat_shard_finish),
                             // and the token word after it (wait_posted)
    unsigned flag_seq = 0;   // the last token posted
    DevBuf app_stat;         // an append's new-row maxima (‖x‖², int8 residual, bf16 residual²)
    hipEvent_t done = nullptr;  // multi-device search: the shard's launch phase has drained (shard 0's stream waits)
};

// What a deferred Flat shard search (flat_shard_search with a FlatPending) leaves to flat_shard_finish: the exact
// forms' flagged queries, whose count is read back into the shard's h_nflag by the launch phase.
struct FlatPending {
    enum Kind { kNone = 0, kSmallI8 = 1, kExact = 2 };
    int kind = kNone;
    int64_t nq = 0;
    const float *xq = nullptr;
    int k = 0, kout = 0;  // k of the re-run (k_user on the batched exact forms), output width
    float *D = nullptr;
    int64_t *I = nullptr;
    // kExact over the bounded passes: the candidate buffers and pass bound for the all-candidate rerank
    const float *cr_d = nullptr, *cr_bound = nullptr;
    const int *cr_i = nullptr, *cr_n = nullptr;
    int cr_nsplit = 0, cr_cap = 0;
    float xmax2 = 0.f, rxmax = 0.f;
    bool i8 = false;
};

struct IndexBase {
    Kind kind;
    int d = 0;
    int metric = kL2;
    std::mutex mu;
    KernelTimer timer_main, timer_merge;
    // the last search's path (hipann_last_search_path): the scan form that ran (FlatForm / IvfForm; an exact
    // form's flagged re-runs excluded), its rerank filter depth (0: no rerank) and sub-lists per slot (IVF)
    int last_form = -1, last_kfilt = 0, last_sublists = 0;
    // per shard, set at create (enable_peer_access): 2 = on shard 0's device (no peer copy), 1 = peer access enabled
    // both ways between its device and shard 0's (the result gather rides xGMI), 0 = not available (the runtime
    // stages the gather through host memory)
    std::vector<int> peer;
    explicit IndexBase(Kind k) : kind(k) {}
    virtual ~IndexBase() = default;
    virtual int64_t ntotal() const = 0;
    virtual int64_t memory_bytes() const = 0;
};

struct FlatIndex : IndexBase {
    std::vector<std::unique_ptr<FlatShard>> shards;
    int form = kFlatI8Exact;  // BLAS-path q·x form (FlatForm); shapes the int8 passes do not take run kFlatBf16Exact
    int64_t rerank_fallbacks = 0;  // queries re-run on the 3-term path by the exact form's bound check
    int64_t cand_reranked = 0;     // form 4: flagged queries sent to the all-candidate rerank first
    int64_t host_syncs = 0;        // host synchronisations in search calls (hipann_flat_host_syncs)
    HostBuf h_q, h_d, h_i;
    DevBuf gather_d, gather_i, merged_d, merged_i;  // multi-device merge on shards[0]'s device
    FlatIndex() : IndexBase(Kind::Flat) {}
    ~FlatIndex() override;
    int64_t ntotal() const override {
        int64_t t = 0;
        for (auto &s : shards) t += s->n;
        return t;
    }
    int64_t memory_bytes() const override {
        int64_t b = 0;
        for (auto &s : shards)
            b += s->n * (int64_t)d * 4 + (metric == kL2 ? s->n * 4 : 0) + (int64_t)s->xb16.bytes +
                 (int64_t)s->xi8.bytes + (int64_t)s->xscale.bytes;
        return b;
    }
};

// IVF: CSR inverted lists resident on one device.  With several devices the lists are partitioned
// (size-balanced); every shard keeps all centroids and an empty range for lists it does not own.
struct IvfShard {
    int device = 0;
    // Physical CSR rows: list l occupies rows [h_off[l], h_off[l+1]) of codes / ids / xnorm, its first h_len[l] live
    // (the rest is append slack, zero-filled; the kernels read list_len, never the gap).  n = h_off[nlist] (the
    // physical row count every whole-table kernel walks), live = Σ h_len (ntotal).
    int64_t n = 0;
    int64_t live = 0;
    const float *centroids = nullptr;
    const float *codes = nullptr;  // n × d fp32, list-contiguous
    const int64_t *ids = nullptr;  // n labels
    DevBuf centroids_buf, codes_buf, ids_buf;  // owned storage (empty when borrowed)
    DevBuf list_off;               // int64 nlist+1 (shard-local physical row offsets: list starts)
    DevBuf list_len;               // int nlist (0 = empty or not owned)
    DevBuf xnorm;                  // ‖x‖² per row (L2; the decomposed scan form)
    std::unique_ptr<FlatIndex> quant;  // coarse quantizer over `centroids` (borrowed)
    hipStream_t stream = nullptr;
    // scratch
    DevBuf q, qn, coarse_d, coarse_i, cnt, bucket_off, item_off, cursor, bucket, slot_off, part_d, part_i, out_d, out_i;
    DevBuf qbound;                 // per query: best known k-th key (order-preserving u32; MFMA scan)
    DevBuf qsplit;                 // split-bf16 scans: the batch's queries as bf16 terms
    // kFormSplit2Exact: max row ‖x‖² (for the rerank's error bound; −1 until computed), the flagged
    // queries of the last batch and the re-run's buffers
    float xmax2 = -1.f;
    DevBuf nflag, flagged, fq, fD, fI, coarse_save, tmpnorm;
    DevBuf ccnt, qtot;             // query-major plan: per-list running counts (kept zero between batches), per-query slot totals
    // the fused plan + fill (ivf_planfill_q): counts and fill cursors double-buffered by batch parity
    // ([2][nlist] each in ccnt / cursor2, zeroed at allocation; each batch zeroes the other parity's pair)
    DevBuf cursor2;
    uint64_t plan_batch = 0;
    int plan_nlist = 0;
    DevBuf fpd, fpi;               // device fallback: per (flagged query, probe) partial lists
    DevBuf fb_total;               // u64 running count of flagged queries (device side)
    DevBuf fbc_d, fbc_i, fbc_done;  // ivf_fallback_chunks: per (flagged query, probe, chunk) lists, per-query counts
    int fbc_cap = 0;               // flagged queries fbc_done holds counters for (zeroed at allocation)
    // MFMA scan copy of the codes, built at the first search that uses it: per list, 32-row passes of
    // [16-dim step][2 row tiles][64 lanes][float4] (ivf_mfma.hip), zero-padded rows / dims
    std::vector<int64_t> h_off;    // host copy of list_off
    std::vector<int64_t> h_len;    // host copy of list_len (live rows per list)
    bool owns_codes = false;       // codes / ids / xnorm in codes_buf / ids_buf (else borrowed: the first add copies)
    DevBuf codes_t, tpass_off;     // tiled codes; int64 nlist+1 pass offsets
    // kFormHalfExact: tiled fp16 image of x·2^half_es (same passes as codes_t), its largest row
    // residual ‖x − x̂·2^−half_es‖ and the batch's query terms / 1/(t·s) / split residuals.
    // half_state: 0 not built, 1 built, −1 unsupported (non-finite or out-of-range codes)
    int half_state = 0, half_es = 0;
    float half_rxmax = 0.f;
    DevBuf codes_h, hsplit, hits, hres;
    // kFormI8Exact: tiled int8 image (same passes), per-row scales, its largest row residual ‖x − s·x̂‖, the batch's
    // int8 queries / scales / residuals; i8_state as half_state (released by appends: rebuilt at the next search)
    int i8_state = 0;
    float i8_rxmax = 0.f;
    DevBuf codes_i8, xs8, qi8, qs8, qres8;
    DevBuf prog;  // fp16 scan: per 64-pass chunk key, the latest item's position (rounds) and the batch it belongs to
    // an append's staging (hipann_ivf_add): the new rows grouped by list, labels, physical destinations, norms,
    // the tiled passes they touch, and the new rows' maxima (‖x‖², |x|, fp16 residual²)
    DevBuf app_rows, app_norm, app_assign, app_up, app_stat;
    DevBuf app_cd;  // hipann_ivf_coarse_device: the coarse distances (discarded)
    // pinned: the assignment on its way down, [destinations | labels | touched passes | live lengths] on their way
    // up (one copy), the maxima on their way down
    HostBuf app_hassign, app_hup[2];
    hipEvent_t app_ev[2] = {nullptr, nullptr};  // app_hup[b]'s upload has been consumed (reused two blocks later)
    hipEvent_t app_sync = nullptr;              // the assignment readback of an append block (polled)
    int app_buf = 0;
    int max_nch = 1;  // largest list's row-chunk count
    StreamFence fence;  // cross-stream ordering of this shard's calls (its coarse quantizer's scratch included)
    hipEvent_t done = nullptr;  // multi-device search: the shard's search has drained (shard 0's stream waits)
};

struct IvfIndex : IndexBase {
    int nlist = 0, nprobe = 1;
    std::vector<int> owner;  // list → shard (size-balanced at create; appended rows follow their list)
    int form = kFormHalfExact;
    int64_t rerank_fallbacks = 0;  // queries re-run from the host (HIPANN_IVF_HOST_FALLBACK); device re-runs: fb_total
    std::vector<std::unique_ptr<IvfShard>> shards;
    int64_t last_nq = 0;
    int last_np = 0;
    HostBuf h_q, h_d, h_i;
    DevBuf gather_d, gather_i, merged_d, merged_i;
    IvfIndex() : IndexBase(Kind::IVF) {}
    ~IvfIndex() override;
    int64_t ntotal() const override {
        int64_t t = 0;
        for (auto &s : shards) t += s->live;
        return t;
    }
    int64_t memory_bytes() const override {
        int64_t b = 0;
        for (auto &s : shards)
            b += s->n * ((int64_t)d * 4 + 8 + (metric == kL2 ? 4 : 0)) + (int64_t)nlist * d * 4 +
                 (int64_t)s->codes_h.bytes + (int64_t)s->codes_t.bytes + (int64_t)s->codes_i8.bytes + (int64_t)s->xs8.bytes;
        return b;
    }
};

// Peer access between every listed device and devs[0] (hipDeviceCanAccessPeer both ways, then
// hipDeviceEnablePeerAccess; an already-enabled pair counts as enabled).  Returns the per-shard state of IndexBase::peer.
std::vector<int> enable_peer_access(const std::vector<int> &devs);

// ---- kernel launchers (flat_kernels.hip, ivf_kernels.hip, ivf_mfma.hip) ----
// host-pointer calls up to this many bytes each way move queries / results with a copy kernel through
// the pinned buffers' device mapping instead of DMA round trips
constexpr size_t kKernelCopyMax = (size_t)64 << 10;
void launch_copy_words(const void *src, void *dst, size_t bytes, hipStream_t st);
// `words` words from device memory to a pinned host buffer (through its device mapping), then `token` into the
// word after them once the copy is visible to the host: the host spins on the token (wait_posted) instead of a
// stream synchronisation.
void launch_post_words(const void *src, void *host_dst, int words, unsigned token, hipStream_t st);
void *host_device_ptr(void *pinned);
void launch_row_norms(const float *x, int64_t n, int d, float *out, hipStream_t st);
size_t gemm_smem_bytes();
void launch_flat_gemm_topk(const float *Q, const float *qn, int64_t nq, const float *X, const float *xn, int64_t N,
                           int d, int metric, int k, int nsplit, int64_t tiles_per_split, float *pd, int *pi,
                           hipStream_t st);
size_t flat_bf_qsplit_bytes(int64_t nq, int d, int np);
void launch_flat_gemm_topk_bf(int np, const float *Q, const float *qn, int64_t nq, void *qsplit, const float *X,
                              const float *xn, int64_t N, int d, int metric, int k, int nsplit, int64_t tiles_per_split,
                              float *pd, int *pi, int qmajor, hipStream_t st);
size_t scan_smem_bytes(int nq, int d);
void launch_flat_gemm_keys(const float *Q, const float *qn, int64_t nq, const float *X, const float *xn, int64_t N,
                           int d, int metric, float *keys, int64_t ldk, hipStream_t st, bool bf3 = false);
void launch_flat_scan_keys(const float *Q, int nq, const float *X, int64_t N, int d, int metric, float *keys,
                           int64_t ldk, hipStream_t st);
void launch_rows_topk(const float *keys, int64_t ldk, int64_t ncols, int64_t nq, int64_t seg_len, int nseg, int k,
                      int id0, float *pd, int *pi, hipStream_t st);
bool launch_rows_select_out(const float *keys, int64_t ldk, int64_t ncols, int64_t nq, int k, int kout,
                            int64_t label_offset, float out_sign, float *D, int64_t *I, hipStream_t st,
                            IvfPlanHook *hook = nullptr);
void launch_merge_raw(const float *pd, const int *pi, int nparts, int64_t nq, int k, float *od, int *oi,
                      hipStream_t st);
void launch_flat_scan_topk(const float *Q, int nq, const float *X, int64_t N, int d, int metric, int k, int nwaves,
                           int64_t rows_per_wave, float *pd, int *pi, hipStream_t st);
void launch_ivf_plan(const int64_t *probes, int64_t nq, int nprobe, const int *list_len, int nlist, int group,
                     int *cnt, int *bucket_off, int *item_off, int *cursor, int *bucket, int *slot_off,
                     hipStream_t st, int *nflag_reset = nullptr, unsigned *qbound = nullptr, int *ccnt = nullptr,
                     int *qtot = nullptr, bool counted = false, int *ccnt_next = nullptr, int *cursor_next = nullptr);
int64_t ivf_max_items(int64_t nq, int nprobe, int nlist, int max_nch, int64_t nrows, int group);
int ivf_mfma_bf_group(int d, int np);
bool ivf_mfma_bf_supported(const float *Q, int d, const float *codes, int k, int np);
int64_t ivf_mfma_bf_qsplit_bytes(int64_t nq, int d, int np);
// Form 4 (bounded passes): the flagged queries' exact top-kout over ALL their buffered candidates, certified
// against the pass bound (every unbuffered row has scan key > bound[q]); queries it cannot certify (a cell
// overflowed, or the k-th distance within the error bound of bound[q]) are appended to flagged2.
void launch_flat_cand_rerank(const int *flagged, int nf, const float *cand_d, const int *cand_i, const int *cand_n,
                             int nsplit, int cap, const float *bound, const float *Q, const float *X, int d,
                             int64_t nrows, int64_t label_offset, float xmax2, float rxmax, int metric, int kout,
                             float *part_d, long long *part_i, int *ovf, float *D, int64_t *I, int *nflag2,
                             int *flagged2, hipStream_t st, float *dbg = nullptr, const float *qres = nullptr);
int flat_cand_rerank_parts(int nsplit);
void launch_ivf_rerank(const float *pd, const int *pi, const int *slot_off, int nprobe, int64_t nq, int k, int kout,
                       int metric, const float *Q, const float *codes, int d, const int64_t *ids, int64_t nrows,
                       int64_t label_offset, float xmax2, float *D, int64_t *I, int *nflag, int *flagged,
                       hipStream_t st, float eps = kSplit2Eps, float rxmax = -1.f, const float *qres = nullptr,
                       const int64_t *probes = nullptr, const int64_t *list_off = nullptr, int nlist = 0,
                       const unsigned *qbound = nullptr, const float *qnorm = nullptr, int kslot = 0, int sub = 0,
                       const int *list_len = nullptr, float *fpd = nullptr, long long *fpi = nullptr,
                       unsigned long long *fb_total = nullptr,  // fpd != nullptr: flagged IVF queries re-run inline
                       int fb_cap = 0);  // ... except the first fb_cap, left to launch_ivf_fallback_chunks
// the rerank's first fb_cap flagged queries re-run in parallel (one wave per (query, probe, chunk) item); cpd/cpi:
// fb_cap·nprobe·maxch·kout entries, done: fb_cap counters (zero on entry; left zero)
void launch_ivf_fallback_chunks(const int *nflag, const int *flagged, int fb_cap, int nprobe, int maxch, int chunk_rows,
                                int kout, int metric, const float *Q, const float *codes, int d, const int64_t *ids,
                                int64_t label_offset, const int64_t *probes, const int64_t *list_off,
                                const int *list_len, int nlist, float *cpd, long long *cpi, unsigned *done, float *D,
                                int64_t *I, unsigned long long *total, hipStream_t st);
// ivf_mfma.hip, fp16-image scan (kFormHalfExact)
int ivf_mfma_h_group(int d);
int ivf_scan_sublists();  // sub-lists per slot of the matrix-core scans in sub-list mode (one per wave)
int64_t ivf_half_pass_bytes(int d);
int64_t ivf_half_qsplit_bytes(int64_t nq, int d);
bool ivf_mfma_h_supported(int d, int k);
void launch_ivf_max_abs(const float *x, int64_t cnt, unsigned *out, hipStream_t st);
// (pass_ids != nullptr: only the listed global passes, one block each — the passes an append touched)
void launch_ivf_tile_half(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                          int nlist, int64_t total_pass, int d, float scale, void *dst, hipStream_t st,
                          const int64_t *pass_ids = nullptr);
void launch_ivf_half_residual(const float *codes, int64_t n, int d, float scale, unsigned *out, hipStream_t st);
void launch_ivf_scan_mfma_h(const float *Q, int64_t nq, void *qsplit, float *its, float *qres, int es, const float *qn,
                            int d, int metric, const void *codes_h, const int64_t *tpass_off, const float *xn,
                            const int64_t *list_off, const int *list_len, const int *cnt, const int *bucket_off, const int *item_off,
                            const int *bucket, const int *slot_off, int nlist, int nprobe, int k, int64_t max_items,
                            unsigned *qbound, float *pd, int *pi, hipStream_t st, bool split_done = false,
                            int sub = 0, unsigned *prog = nullptr, int nprog = 0, unsigned epoch = 0, int i8mode = 0,
                            const float *xs8 = nullptr);
// int8 image (kFormI8Exact): packed group (wide items only), pass / query-image bytes, support, the tiling (one scale per
// row into xs8), max row residual² (float bits), the batch's int8 queries (units, scales, residuals)
int ivf_mfma_i8_group(int d);
int64_t ivf_i8_pass_bytes(int d);
int64_t ivf_i8_qimg_bytes(int64_t nq, int d);
bool ivf_mfma_i8_supported(int d, int k);
void launch_ivf_tile_i8(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                        int nlist, int64_t total_pass, int d, void *dst, float *xs8, hipStream_t st,
                        const int64_t *pass_ids = nullptr);
void launch_ivf_i8_residual(const float *codes, int64_t n, int d, unsigned *out, hipStream_t st);
void launch_ivf_split_queries_i8(const float *Q, int64_t nq, int d, void *qi8, float *qs8, float *qres8,
                                 hipStream_t st);
// the batch's fp16 query terms (+ 1/(t·s), split residuals) and, when qn != nullptr, ‖q‖² (row_norms_f32's bits)
void launch_ivf_split_queries_h(const float *Q, int64_t nq, int d, int es, void *qsplit, float *its, float *qres,
                                float *qn, hipStream_t st);
// flat_bf16.hip
int flat_bf16_waves(int64_t nq);
int flat_bf16_tile_rows();
int flat_bf16_topk_kmax(int64_t nq);
int flat_gemm_topk_bf_kmax(int np);
size_t flat_bf16_img_bytes(int64_t n, int d, int R);
void launch_b16_tile_rows(const float *X, int64_t n, int d, int R, void *out, hipStream_t st);
void launch_b16_row_residual2(const float *X, int64_t n, int d, float *out, hipStream_t st);
void launch_flat_bf16_topk(const float *Q, const float *qn, int64_t nq, void *qimg, const void *ximg, const float *xn,
                           int64_t N, int d, int metric, int k, int nsplit, int64_t tiles_per_split, float *pd, int *pi,
                           const float *seed, bool image_ready, hipStream_t st);
// bounded passes of the 64-dim K-step kernel (flat_b16k64.hip): candidate buffers, their bound and select
bool flat_bf16_resumable(int64_t nq, int d, int k);
void launch_flat_bf16_k64(const void *qimg, const float *qn, int64_t nq, const void *ximg, const float *xn, int64_t N,
                          int nk, int metric, int nqt, int nsplit, int64_t tiles_per_split, int64_t tile_begin,
                          int64_t tile_end, const float *bound, float *cand_d, int *cand_i, int *cand_n, int cap,
                          bool resume, bool keys, hipStream_t st, const float *qscale = nullptr,
                          const float *xscale = nullptr);
// form kFlatI8Exact (flat_b16k64.hip): per-row int8 scale s = max|x|/127 and residual ‖x − s·x̂‖ (×1.0001) per row;
// the tiled int8 image (64 dims per 64-B chunk row, chunk count rounded up to even, zero-filled); its bytes
int flat_i8_nk(int d);
size_t flat_i8_img_bytes(int64_t n, int d, int R);
void launch_i8_row_scale(const float *X, int64_t n, int d, float *scale, float *resid, hipStream_t st);
void launch_i8_tile_rows(const float *X, const float *scale, int64_t n, int d, int R, void *out, hipStream_t st);
// ‖q‖² (qn optional), the int8 scales / residuals and the tiled int8 image of a query batch in one launch
void launch_i8_query_prep(const float *X, int64_t n, int d, float *qn, float *scale, float *resid, int R, void *out,
                          hipStream_t st);
int flat_i8_scan_k();
int flat_i8_scan_max_nq();
int64_t flat_i8_scan_waves(int64_t n);
void launch_flat_i8_scan(const float *Q, int64_t nq, int d, int metric, const void *ximg, const float *xscale,
                         const float *xnorm, int64_t n, float *qscale, float *qres, const float *qnorm, void *qimg,
                         float *part_d, int *part_i, int64_t nw, hipStream_t st);
void launch_flat_i8_group_merge(const float *pd, const int *pi, int nw, int nq, int ngroup, float *od, int *oi,
                                hipStream_t st);
int flat_keys_kth_max();
void launch_flat_keys_kth(const float *keys, int S, int64_t nq, int k, float *bound, hipStream_t st);
void launch_flat_cand_bound(const float *cand_d, const int *cand_n, int nsplit, int cap, int64_t nq, int k,
                            float *bound, hipStream_t st);
void launch_flat_cand_select(const float *cand_d, const int *cand_i, const int *cand_n, int nsplit, int cap, int64_t nq,
                             int k, float *out_d, int *out_i, int *nflag, int *flagged, hipStream_t st);
void launch_flat_bf16_seed(const float *pd, int nsplit, int64_t nq, int k, float *seed, hipStream_t st);
bool flat_bf16_k64_supported(int nk, int k);
void launch_ivf_max_norm(const float *xn, int64_t n, unsigned *out, hipStream_t st);
void launch_ivf_gather_queries(const float *Q, const int *idx, int nf, int d, float *out, hipStream_t st);
// hipann_ivf_add: an append block's rows into their CSR rows + the new live lengths + the new rows' maxima
// (stat[0] max ‖x‖², stat[1] max |x| bits, stat[2] max fp16 residual² at hscale; hscale 0: no residual)
void launch_ivf_append_rows(const float *rows, const float *norms, const int64_t *dst, const int64_t *ids_in, int64_t n,
                            int d, float *codes, int64_t *ids, float *xnorm, const int *newlen, int *list_len, int nlist,
                            float hscale, unsigned *stat, hipStream_t st);
void launch_ivf_scatter_results(const float *Df, const int64_t *If, const int *idx, int nf, int kout, float *D,
                                int64_t *I, hipStream_t st);
void launch_ivf_scan_mfma_bf(int np, const float *Q, int64_t nq, void *qsplit, const float *qn, int d, int metric,
                             const float *codes_t, const int64_t *tpass_off, const float *xn, const int64_t *list_off,
                             const int *list_len, const int *cnt, const int *bucket_off, const int *item_off, const int *bucket,
                             const int *slot_off, int nlist, int nprobe, int k, int64_t max_items, unsigned *qbound,
                             float *pd, int *pi, hipStream_t st, int sub = 0);
int ivf_group_size(int form, int d);  // queries per work item of the form's scan kernel
int ivf_chunk_rows();
bool ivf_plan_query_major();
void launch_ivf_scan_bigk(const float *Q, int d, int metric, const float *codes, const int64_t *list_off,
                          const int *list_len, const int64_t *probes, int64_t npairs, int nprobe, const int *slot_off, int64_t nslots,
                          int k, float *pd, int *pi, hipStream_t st);
size_t ivf_scan_smem_bytes();
bool ivf_dot_supported(const float *Q, int d, const float *codes);
void launch_ivf_scan(const float *Q, const float *qn, int d, int metric, int form, const float *codes,
                     const float *xn, const int64_t *list_off, const int *list_len, const int *cnt,
                     const int *bucket_off, const int *item_off, const int *bucket, const int *slot_off, int nlist,
                     int nprobe, int64_t nq,
                     int k, int64_t max_items, unsigned *qbound, float *pd, int *pi, hipStream_t st);
bool ivf_mfma_supported(const float *Q, int d, const float *codes, int k);
int ivf_mfma_group(int d);
int64_t ivf_mfma_pass_floats(int d);  // floats per 32-row pass of the tiled codes
void launch_ivf_tile_codes(const float *codes, const int64_t *list_off, const int *list_len, const int64_t *tpass_off,
                           int nlist, int64_t total_pass, int d, float *dst, hipStream_t st,
                           const int64_t *pass_ids = nullptr);
void launch_ivf_scan_mfma(const float *Q, const float *qn, int d, int metric, const float *codes_t,
                          const int64_t *tpass_off, const float *xn,
                          const int64_t *list_off, const int *list_len, const int *cnt, const int *bucket_off, const int *item_off,
                          const int *bucket, const int *slot_off, int nlist, int nprobe, int k, int64_t max_items,
                          unsigned *qbound, float *pd, int *pi, hipStream_t st, int sub = 0);
void launch_ivf_merge(const float *pd, const int *pi, const int64_t *ids, int64_t nrows, const int *slot_off, int nprobe, int64_t nq,
                      int k, int kout, float out_sign, float *D, int64_t *I, hipStream_t st);
template <typename InId>
void launch_merge_parts(const float *pd, const InId *pi, int nparts, int64_t nq, int k, int kout,
                        int64_t label_offset, float in_sign, float out_sign, float *D, int64_t *I, hipStream_t st,
                        int64_t pstride_d = -1, int64_t pstride_i = -1);  // part strides (elements); -1: nq*k
// Many parts, few queries: groups of parts merged by ngroups·nq waves into md/mi ([g][nq][kout]), then the
// group lists by launch_merge_parts (kout <= 64).
template <typename InId>
void launch_merge_parts_2level(const float *pd, const InId *pi, int nparts, int64_t nq, int k, int kout,
                               int64_t label_offset, float in_sign, float out_sign, float *D, int64_t *I, float *md,
                               long long *mi, int ngroups, hipStream_t st);

}  // namespace hipann
