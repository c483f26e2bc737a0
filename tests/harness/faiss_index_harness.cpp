// faiss_index_harness.cpp — TEST PROGRAM (not product code): the extension's FaissIndex search/upload flow
// restated over the C ABI (include/hip_ann.h), with the SURVEY §8f rank 1 and rank 2 changes applied.
//
// The reference cannot be compiled here (no DuckDB, no FAISS), so this program restates the parts of
// src/faiss_index.cpp that drive the GPU copy, line for line in behaviour:
//   FaissIndex::EnsureGpuIndex      faiss_index.cpp:108-149 (mode CPU / GPU / AUTO; AUTO gate = the MI355X
//                                   HIPANN_AUTO_MIN_WORK of hip_ann.h instead of ntotal >= 256 && d >= 128)
//   FaissIndex::InvalidateGpuIndex  :151-153
//   FaissIndex::Append              :430-472 (labels ntotal + i, label↔rowid maps) — rank 2: the rows are
//                                   appended to the GPU copy (hipann_flat_add / hipann_ivf_add) instead of :469
//   FaissIndex::Delete              :478-500 (tombstones)
//   FaissIndex::Vacuum              :840-899 (compaction, relabel, invalidate) — rank 2: the next Search
//                                   re-uploads lazily
//   FaissIndex::Search              :708-762 (request_k = min(k + |deleted|, ntotal), nprobe, search(1, …),
//                                   −1 / tombstone skip, label → rowid)
//   FaissIndex::SearchBatch         rank 1: the same rules, ONE search(nq, …) call
//   PhysicalCreateFaissIndex::Finalize training (:302-319) and the Vacuum retrain (:876-878) — INTEGRATION.md
//                                   §1.4: IVF k-means on the GPU (hipann_ivf_train) when the mode is not CPU;
//                                   the CPU twin trains with the oracle's restatement (same draws)
// The "CPU FAISS index" is the oracle's restatement of IndexFlat / IndexIVFFlat (oracle/oracle.c, test
// infrastructure); the "GPU index" is libhipann.so.  Every scenario compares the GPU-backed FaissIndex with a
// CPU-mode twin fed the same operations.  Output: one "CHECK <name> ok|FAIL <detail>" line per check, exit
// status 0 iff every check passed.  Driven by tests/test_harness_gpu.py.
#include "../../include/hip_ann.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

extern "C" {  // oracle/oracle.c (liboracle.so)
void oracle_flat_search(const float *xb, int64_t n, int d, const float *xq, int64_t nq, int k, int metric,
                        int64_t label_offset, float *D, int64_t *I);
void oracle_ivf_search(const float *centroids, int nlist, const int64_t *list_off, const int64_t *ids,
                       const float *codes, int d, const float *xq, int64_t nq, int k, int nprobe, int metric, float *D,
                       int64_t *I, int64_t *probes_out);
int oracle_kmeans_train(const float *x, int64_t n, int d, int metric, int nlist, int64_t train_sample, int niter,
                        uint64_t seed, int init, float *centroids, int64_t *sizes_out);
}

namespace {

using row_t = int64_t;
using Result = std::vector<std::pair<row_t, float>>;

int g_fail = 0;
void check(bool ok, const std::string &name, const std::string &detail = "") {
    std::printf("CHECK %s %s%s%s\n", name.c_str(), ok ? "ok" : "FAIL", detail.empty() ? "" : " ", detail.c_str());
    if (!ok) ++g_fail;
}

// ---- the CPU FAISS index (IndexFlat / IndexIVFFlat), restated by the oracle ---------------------------
struct CpuIndex {
    int d = 0, metric = 0;
    bool ivf = false;
    int nlist = 0;
    std::vector<float> rows;                      // Flat: ntotal × d in label order
    std::vector<float> centroids;                 // IVF: trained coarse quantizer
    std::vector<std::vector<int64_t>> list_ids;   // IVF: ArrayInvertedLists
    std::vector<std::vector<float>> list_codes;
    std::vector<float> by_label;                  // every vector by label (reconstruct_n for Vacuum / Merge)
    int64_t ntotal = 0;

    // IndexIVF::add_with_ids → quantizer->assign (k = 1) → append to the list in insertion order
    void add(int64_t n, const float *x) {
        by_label.insert(by_label.end(), x, x + n * d);
        if (!ivf) {
            rows.insert(rows.end(), x, x + n * d);
        } else {
            std::vector<float> dd(n);
            std::vector<int64_t> a(n);
            for (int64_t i0 = 0; i0 < n; i0 += 65536) {  // FAISS assigns in blocks of 65536 rows
                const int64_t m = std::min<int64_t>(65536, n - i0);
                oracle_flat_search(centroids.data(), nlist, d, x + i0 * d, m, 1, metric, 0, dd.data() + i0,
                                   a.data() + i0);
            }
            for (int64_t i = 0; i < n; ++i) {
                list_ids[a[i]].push_back(ntotal + i);
                list_codes[a[i]].insert(list_codes[a[i]].end(), x + i * d, x + (i + 1) * d);
            }
        }
        ntotal += n;
    }
    void csr(std::vector<int64_t> &off, std::vector<int64_t> &ids, std::vector<float> &codes) const {
        off.assign(nlist + 1, 0);
        ids.clear();
        codes.clear();
        for (int l = 0; l < nlist; ++l) {
            off[l + 1] = off[l] + (int64_t)list_ids[l].size();
            ids.insert(ids.end(), list_ids[l].begin(), list_ids[l].end());
            codes.insert(codes.end(), list_codes[l].begin(), list_codes[l].end());
        }
    }
    void search(int64_t nq, const float *x, int k, int nprobe, float *D, int64_t *I) const {
        if (!ivf) {
            oracle_flat_search(rows.data(), ntotal, d, x, nq, k, metric, 0, D, I);
            return;
        }
        std::vector<int64_t> off, ids;
        std::vector<float> codes;
        csr(off, ids, codes);
        oracle_ivf_search(centroids.data(), nlist, off.data(), ids.data(), codes.data(), d, x, nq, k, nprobe, metric, D,
                          I, nullptr);
    }
};

enum class Mode { CPU, GPU, AUTO };

// ---- the FaissIndex BoundIndex, restated ---------------------------------------------------------------
struct FaissIndexModel {
    int dimension_ = 0, metric_ = 0, nprobe_ = 1;
    std::string index_type_;
    Mode mode_ = Mode::AUTO;
    std::unique_ptr<CpuIndex> faiss_index_;
    void *gpu_index_ = nullptr;
    std::vector<row_t> label_to_rowid_;
    std::unordered_map<row_t, int64_t> rowid_to_label_;
    std::unordered_set<int64_t> deleted_labels_;
    int uploads = 0;        // CpuToGpu calls (EnsureGpuIndex uploads)
    int gpu_appends = 0;    // rows appended to the GPU copy (rank 2)
    int gpu_searches = 0;   // search() calls served by the GPU copy

    ~FaissIndexModel() { InvalidateGpuIndex(); }

    void InvalidateGpuIndex() {  // faiss_index.cpp:151-153
        if (gpu_index_) hipann_free(gpu_index_);
        gpu_index_ = nullptr;
    }

    // GpuBackend::CpuToGpu (gpu_backend_metal.mm:42-60 → adapters/gpu_backend_hip.cpp): IVFFlat first, then Flat
    void *CpuToGpu() {
        char err[512] = {0};
        const CpuIndex &c = *faiss_index_;
        void *h = nullptr;
        if (c.ivf) {
            std::vector<int64_t> off, ids;
            std::vector<float> codes;
            c.csr(off, ids, codes);
            h = hipann_ivf_create(c.d, c.metric, c.nlist, nprobe_, c.centroids.data(), off.data(), ids.data(),
                                  codes.data(), nullptr, 0, err, sizeof err);
        } else {
            h = hipann_flat_create(c.d, c.metric, c.rows.data(), c.ntotal, nullptr, 0, err, sizeof err);
        }
        if (!h) throw std::runtime_error(err);
        ++uploads;
        return h;
    }

    void EnsureGpuIndex() {  // faiss_index.cpp:108-149
        if (mode_ == Mode::CPU || !faiss_index_ || gpu_index_) return;
        if (mode_ == Mode::GPU) {
            if (!hipann_available()) throw std::invalid_argument("mode='gpu' requested but no GPU backend available");
            gpu_index_ = CpuToGpu();
            return;
        }
        if (!hipann_available()) return;
        if (index_type_ == "HNSW" || index_type_ == "hnsw") return;
        // MI355X AUTO gate (replaces ntotal < 256 || dimension_ < 128, :136-143)
        if (faiss_index_->ntotal * (int64_t)dimension_ < HIPANN_AUTO_MIN_WORK) return;
        try {
            gpu_index_ = CpuToGpu();
        } catch (std::runtime_error &) {
        }
    }

    // IVF training: GPU k-means when a GPU may serve, the CPU train otherwise.  Both take
    // the reference's stride sample of train_sample rows (:304-315) and the same seed.
    static constexpr int kTrainIters = 25;
    static constexpr uint64_t kTrainSeed = 1234;
    int gpu_trains = 0;
    void Train(const float *x, int64_t n, int64_t train_sample) {
        CpuIndex &c = *faiss_index_;
        if (!c.ivf || n <= 0) return;
        c.centroids.assign((size_t)c.nlist * c.d, 0.f);
        if (mode_ != Mode::CPU && hipann_available()) {
            char err[512] = {0};
            const int rc = hipann_ivf_train(c.d, c.metric, c.nlist, n, x, train_sample, kTrainIters, kTrainSeed,
                                            HIPANN_KMEANS_INIT_RANDOM, 0, c.centroids.data(), nullptr, err, sizeof err);
            if (rc == 0) {
                ++gpu_trains;
                return;
            }
            if (mode_ == Mode::GPU) throw std::runtime_error(err);
        }
        if (oracle_kmeans_train(x, n, c.d, c.metric, c.nlist, train_sample, kTrainIters, kTrainSeed,
                                HIPANN_KMEANS_INIT_RANDOM, c.centroids.data(), nullptr) != 0)
            throw std::runtime_error("CPU training failed");
    }

    // Finalize (:287-414): train (IVF), add, label↔rowid maps, EnsureGpuIndex (:364)
    void Finalize(const std::vector<float> &x, const std::vector<row_t> &rowids, int64_t train_sample = -1) {
        if (train_sample >= 0) Train(x.data(), (int64_t)rowids.size(), train_sample);
        faiss_index_->add((int64_t)rowids.size(), x.data());
        for (size_t i = 0; i < rowids.size(); ++i) {
            label_to_rowid_.push_back(rowids[i]);
            rowid_to_label_[rowids[i]] = (int64_t)i;
        }
        EnsureGpuIndex();
    }

    void Append(const std::vector<float> &x, const std::vector<row_t> &rowids) {  // :430-472
        const int64_t count = (int64_t)rowids.size();
        if (!count) return;
        const int64_t base_label = faiss_index_->ntotal;
        faiss_index_->add(count, x.data());
        if (base_label + count > (int64_t)label_to_rowid_.size()) label_to_rowid_.resize(base_label + count, -1);
        for (int64_t i = 0; i < count; ++i) {
            label_to_rowid_[base_label + i] = rowids[i];
            rowid_to_label_[rowids[i]] = base_label + i;
        }
        // SURVEY §8f rank 2 (replaces InvalidateGpuIndex() at :469): append to the GPU copy, same labels
        if (gpu_index_) {
            char err[512] = {0};
            const bool ivf = faiss_index_->ivf;
            std::vector<int64_t> labels(count);
            for (int64_t i = 0; i < count; ++i) labels[i] = base_label + i;
            const int rc = ivf ? hipann_ivf_add(gpu_index_, count, x.data(), labels.data(), err, sizeof err)
                               : hipann_flat_add(gpu_index_, x.data(), count, err, sizeof err);
            if (rc != 0) InvalidateGpuIndex();
            else gpu_appends += (int)count;
        }
    }

    void Delete(const std::vector<row_t> &rowids) {  // :478-500
        for (row_t r : rowids) {
            auto it = rowid_to_label_.find(r);
            if (it != rowid_to_label_.end()) {
                deleted_labels_.insert(it->second);
                rowid_to_label_.erase(it);
            }
        }
    }

    void Vacuum(bool retrain = false) {  // :840-899; retrain: the fresh IVF index is trained on every kept row (:876-878)
        if (deleted_labels_.empty() || !faiss_index_) return;
        const int64_t old_ntotal = faiss_index_->ntotal;
        std::vector<float> kept;
        std::vector<row_t> kept_rowids;
        for (int64_t i = 0; i < old_ntotal; ++i) {
            if (deleted_labels_.count(i)) continue;
            kept.insert(kept.end(), faiss_index_->by_label.begin() + i * dimension_,
                        faiss_index_->by_label.begin() + (i + 1) * dimension_);
            if (i < (int64_t)label_to_rowid_.size()) kept_rowids.push_back(label_to_rowid_[i]);
        }
        auto fresh = std::make_unique<CpuIndex>();
        fresh->d = faiss_index_->d;
        fresh->metric = faiss_index_->metric;
        fresh->ivf = faiss_index_->ivf;
        fresh->nlist = faiss_index_->nlist;
        fresh->centroids = faiss_index_->centroids;
        fresh->list_ids.assign(fresh->nlist, {});
        fresh->list_codes.assign(fresh->nlist, {});
        std::swap(faiss_index_, fresh);
        if (retrain && !kept_rowids.empty()) Train(kept.data(), (int64_t)kept_rowids.size(), 0);
        std::swap(faiss_index_, fresh);
        if (!kept_rowids.empty()) fresh->add((int64_t)kept_rowids.size(), kept.data());
        label_to_rowid_.assign(kept_rowids.begin(), kept_rowids.end());
        rowid_to_label_.clear();
        for (size_t i = 0; i < kept_rowids.size(); ++i) rowid_to_label_[kept_rowids[i]] = (int64_t)i;
        faiss_index_ = std::move(fresh);
        deleted_labels_.clear();
        InvalidateGpuIndex();
    }

    // search(n, x, k, D, I) on whichever copy serves (:729, :737); nprobe per call (:720-726 sets it on the CPU
    // index; the GPU copy takes it per call under its lock — hipann_ivf_search_np)
    void index_search(int64_t n, const float *x, int k, float *D, int64_t *I) {
        if (gpu_index_) {
            char err[512] = {0};
            const int rc = faiss_index_->ivf
                               ? hipann_ivf_search_np(gpu_index_, nprobe_, n, x, k, D, I, err, sizeof err)
                               : hipann_flat_search(gpu_index_, n, x, k, D, I, err, sizeof err);
            if (rc != 0) throw std::runtime_error(err);
            ++gpu_searches;
            return;
        }
        faiss_index_->search(n, x, k, nprobe_, D, I);
    }

    int32_t request_k(int32_t k) const {  // :713-716
        int64_t r = (int64_t)k + (int64_t)deleted_labels_.size();
        r = std::min<int64_t>(r, faiss_index_->ntotal);
        return (int32_t)std::min<int64_t>(r, INT32_MAX);
    }

    void collect(const float *D, const int64_t *I, int32_t rk, int32_t k, Result &out) const {  // :745-759
        out.clear();
        for (int32_t i = 0; i < rk && (int32_t)out.size() < k; ++i) {
            const int64_t label = I[i];
            if (label < 0) continue;
            if (deleted_labels_.count(label)) continue;
            if (label < (int64_t)label_to_rowid_.size()) out.emplace_back(label_to_rowid_[label], D[i]);
        }
    }

    Result Search(const float *query, int32_t dimension, int32_t k) {  // :708-762
        if (!faiss_index_ || dimension != dimension_) return {};
        const int32_t rk = request_k(k);
        if (rk <= 0) return {};
        if (!gpu_index_ && mode_ != Mode::CPU) EnsureGpuIndex();  // rank 2: lazy re-upload after invalidation
        std::vector<float> D(rk);
        std::vector<int64_t> I(rk);
        index_search(1, query, rk, D.data(), I.data());
        Result out;
        collect(D.data(), I.data(), rk, k, out);
        return out;
    }

    std::vector<Result> SearchBatch(const float *queries, int64_t nq, int32_t dimension, int32_t k) {  // rank 1
        std::vector<Result> out(nq > 0 ? nq : 0);
        if (!faiss_index_ || dimension != dimension_ || nq <= 0) return out;
        const int32_t rk = request_k(k);
        if (rk <= 0) return out;
        if (!gpu_index_ && mode_ != Mode::CPU) EnsureGpuIndex();
        std::vector<float> D((size_t)nq * rk);
        std::vector<int64_t> I((size_t)nq * rk);
        index_search(nq, queries, rk, D.data(), I.data());  // one call for the whole batch
        for (int64_t q = 0; q < nq; ++q) collect(D.data() + q * rk, I.data() + q * rk, rk, k, out[q]);
        return out;
    }
};

std::unique_ptr<FaissIndexModel> make_model(const std::string &type, int d, int metric, Mode mode, int nlist,
                                            const std::vector<float> &centroids, int nprobe) {
    auto m = std::make_unique<FaissIndexModel>();
    m->dimension_ = d;
    m->metric_ = metric;
    m->index_type_ = type;
    m->mode_ = mode;
    m->nprobe_ = nprobe;
    m->faiss_index_ = std::make_unique<CpuIndex>();
    m->faiss_index_->d = d;
    m->faiss_index_->metric = metric;
    if (type == "IVFFlat") {
        m->faiss_index_->ivf = true;
        m->faiss_index_->nlist = nlist;
        m->faiss_index_->centroids = centroids;
        m->faiss_index_->list_ids.assign(nlist, {});
        m->faiss_index_->list_codes.assign(nlist, {});
    }
    return m;
}

// Results equal: same rowids in the same order; distances within rtol (the GPU's exact forms return FAISS's
// fp32 distances up to summation order).
bool same(const Result &a, const Result &b, double rtol, std::string *why) {
    if (a.size() != b.size()) {
        if (why) *why = "sizes " + std::to_string(a.size()) + " vs " + std::to_string(b.size());
        return false;
    }
    for (size_t i = 0; i < a.size(); ++i) {
        if (a[i].first != b[i].first) {
            if (why) *why = "rank " + std::to_string(i) + ": rowid " + std::to_string(a[i].first) + " vs " +
                            std::to_string(b[i].first);
            return false;
        }
        const double x = a[i].second, y = b[i].second;
        if (std::fabs(x - y) > rtol * std::max(1.0, std::fabs(y))) {
            if (why) *why = "rank " + std::to_string(i) + ": dist " + std::to_string(x) + " vs " + std::to_string(y);
            return false;
        }
    }
    return true;
}

int count_diff(const std::vector<Result> &a, const std::vector<Result> &b, double rtol, std::string *first) {
    int n = 0;
    for (size_t q = 0; q < a.size(); ++q) {
        std::string why;
        if (!same(a[q], b[q], rtol, &why)) {
            if (!n && first) *first = "query " + std::to_string(q) + " " + why;
            ++n;
        }
    }
    return n;
}

std::vector<float> uniform(std::mt19937 &rng, int64_t n) {  // faiss-metal's test inputs: U(-1, 1)
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<float> v((size_t)n);
    for (auto &x : v) x = u(rng);
    return v;
}

// One scenario: a GPU-mode (or AUTO) FaissIndex and its CPU-mode twin through build → search → delete →
// append → search → vacuum → lazy re-upload → search.
void scenario(const std::string &type, int d, int metric, int64_t n, int nq, int k, int nlist, int nprobe,
              Mode mode, int64_t train_sample = -1) {
    // train_sample >= 0: the IVF quantizer is trained at Finalize (and again at Vacuum) — §1.4
    const bool train = type == "IVFFlat" && train_sample >= 0;
    const std::string tag = type + (metric ? "_ip" : "_l2") + "_d" + std::to_string(d) + (train ? "_trained" : "");
    std::mt19937 rng(42);
    std::vector<float> xb = uniform(rng, n * d), xq = uniform(rng, (int64_t)nq * d);
    std::vector<float> cen;
    if (type == "IVFFlat" && !train)  // a given quantizer: every (n / nlist)-th row
        for (int l = 0; l < nlist; ++l) cen.insert(cen.end(), xb.begin() + (int64_t)l * (n / nlist) * d,
                                                  xb.begin() + ((int64_t)l * (n / nlist) + 1) * d);
    std::vector<row_t> rowids(n);
    for (int64_t i = 0; i < n; ++i) rowids[i] = 1000000 + 7 * i;  // DuckDB row ids, not labels
    auto gpu = make_model(type, d, metric, mode, nlist, cen, nprobe);
    auto cpu = make_model(type, d, metric, Mode::CPU, nlist, cen, nprobe);
    gpu->Finalize(xb, rowids, train ? train_sample : -1);
    cpu->Finalize(xb, rowids, train ? train_sample : -1);
    if (train) {
        check(gpu->gpu_trains == 1 && cpu->gpu_trains == 0, tag + "/finalize/trained_on_gpu");
        check(gpu->faiss_index_->centroids == cpu->faiss_index_->centroids, tag + "/finalize/centroids_equal_cpu_train");
    }
    check(gpu->gpu_index_ != nullptr && gpu->uploads == 1, tag + "/finalize_uploads");
    check(cpu->gpu_index_ == nullptr && cpu->uploads == 0, tag + "/cpu_mode_never_uploads");

    auto run = [&](const std::string &step) {
        // SearchBatch (one GPU call) == CPU path; Search(1) loop == CPU path; SearchBatch == Search loop
        std::vector<Result> gb = gpu->SearchBatch(xq.data(), nq, d, k), cb = cpu->SearchBatch(xq.data(), nq, d, k);
        std::vector<Result> gs(nq), cs(nq);
        for (int q = 0; q < nq; ++q) {
            gs[q] = gpu->Search(xq.data() + (int64_t)q * d, d, k);
            cs[q] = cpu->Search(xq.data() + (int64_t)q * d, d, k);
        }
        std::string w1, w2, w3;
        const int d1 = count_diff(gb, cb, 2e-5, &w1), d2 = count_diff(gs, cs, 2e-5, &w2),
                  d3 = count_diff(gb, gs, 2e-5, &w3);
        check(d1 == 0, tag + "/" + step + "/search_batch_equals_cpu_path", d1 ? std::to_string(d1) + " queries; " + w1 : "");
        check(d2 == 0, tag + "/" + step + "/search_equals_cpu_path", d2 ? std::to_string(d2) + " queries; " + w2 : "");
        check(d3 == 0, tag + "/" + step + "/search_batch_equals_search_loop", d3 ? std::to_string(d3) + " queries; " + w3 : "");
        size_t full = 0;
        for (auto &r : gb) full += r.size() == (size_t)k;
        check(full == (size_t)nq, tag + "/" + step + "/k_results_per_query");
        return gb;
    };
    const int before = gpu->gpu_searches;
    std::vector<Result> r0 = run("built");
    check(gpu->gpu_searches - before == 1 + nq, tag + "/built/served_by_gpu_copy");

    // tombstones: delete the current top-1 of every query (and a stride of others)
    std::vector<row_t> del;
    for (auto &r : r0)
        if (!r.empty()) del.push_back(r[0].first);
    for (int64_t i = 0; i < n; i += 97) del.push_back(rowids[i]);
    gpu->Delete(del);
    cpu->Delete(del);
    std::vector<Result> r1 = run("deleted");
    std::set<row_t> dset(del.begin(), del.end());
    bool none = true;
    for (auto &r : r1)
        for (auto &p : r) none = none && !dset.count(p.first);
    check(none, tag + "/deleted/tombstones_skipped");
    check(gpu->uploads == 1, tag + "/deleted/no_reupload");

    // append: the rows land on the GPU copy (no invalidation, no re-upload); an appended row finds itself
    const int64_t na = n / 4;
    std::vector<float> xa = uniform(rng, na * d);
    std::vector<row_t> ra(na);
    for (int64_t i = 0; i < na; ++i) ra[i] = 9000000 + i;
    void *h_before = gpu->gpu_index_;
    gpu->Append(xa, ra);
    cpu->Append(xa, ra);
    check(gpu->gpu_index_ == h_before && gpu->uploads == 1 && gpu->gpu_appends == na, tag + "/append/on_gpu_copy",
          "uploads=" + std::to_string(gpu->uploads) + " appended=" + std::to_string(gpu->gpu_appends));
    check(hipann_ntotal(gpu->gpu_index_) == n + na, tag + "/append/ntotal");
    run("appended");
    if (metric == 0) {
        Result self = gpu->Search(xa.data() + 5 * d, d, k);
        check(!self.empty() && self[0].first == ra[5] && self[0].second == 0.f, tag + "/append/self_query_first");
    }

    // vacuum: relabels → the copy is dropped; the next search re-uploads it once (rank 2's lazy re-upload)
    gpu->Vacuum(train);
    cpu->Vacuum(train);
    if (train) {
        check(gpu->gpu_trains == 2, tag + "/vacuum/retrained_on_gpu");
        check(gpu->faiss_index_->centroids == cpu->faiss_index_->centroids, tag + "/vacuum/centroids_equal_cpu_train");
    }
    check(gpu->gpu_index_ == nullptr, tag + "/vacuum/invalidated");
    run("vacuumed");
    check(gpu->gpu_index_ != nullptr && gpu->uploads == 2, tag + "/vacuum/lazy_reupload_once",
          "uploads=" + std::to_string(gpu->uploads));
    check(hipann_ntotal(gpu->gpu_index_) == cpu->faiss_index_->ntotal, tag + "/vacuum/ntotal");

    // wrong dimension → no rows (faiss_basic.test:262-269); k > ntotal → ntotal rows
    check(gpu->Search(xq.data(), d + 1, k).empty(), tag + "/wrong_dimension_empty");
}

}  // namespace

int main() {
    if (!hipann_available()) {
        std::printf("CHECK device FAIL no gfx950 HIP device\n");
        return 2;
    }
    char info[256] = {0};
    hipann_device_info(info, sizeof info);
    std::printf("device %s\n", info);
    // Flat: AUTO mode (ntotal·d above the MI355X gate) and explicit GPU mode; L2 and IP; IVFFlat with nprobe < nlist
    scenario("Flat", 128, 0, 20000, 64, 10, 0, 1, Mode::AUTO);
    scenario("Flat", 96, 1, 12000, 40, 10, 0, 1, Mode::GPU);
    scenario("IVFFlat", 64, 0, 30000, 48, 10, 32, 8, Mode::GPU);
    scenario("IVFFlat", 64, 1, 30000, 48, 10, 32, 8, Mode::GPU);
    // CREATE INDEX training on the GPU (§1.4): stride sample of 6000 rows; the VACUUM retrain uses every kept row
    scenario("IVFFlat", 64, 0, 30000, 48, 10, 32, 8, Mode::GPU, 6000);
    scenario("IVFFlat", 48, 1, 24000, 40, 10, 24, 6, Mode::AUTO, 0);
    // AUTO below the gate stays on the CPU (ntotal·d < HIPANN_AUTO_MIN_WORK)
    {
        std::mt19937 rng(7);
        std::vector<float> xb = uniform(rng, 512 * 128);
        std::vector<row_t> rid(512);
        for (int i = 0; i < 512; ++i) rid[i] = i;
        auto m = make_model("Flat", 128, 0, Mode::AUTO, 0, {}, 1);
        m->Finalize(xb, rid);
        check(m->gpu_index_ == nullptr, "auto_gate/small_table_stays_on_cpu");
        Result r = m->Search(xb.data(), 128, 5);
        check(!r.empty() && r[0].first == 0, "auto_gate/cpu_search_works");
        // k > ntotal: request_k clamps to ntotal (edge_cases.test:99-105)
        auto g = make_model("Flat", 128, 0, Mode::GPU, 0, {}, 1);
        std::vector<float> x3(xb.begin(), xb.begin() + 3 * 128);
        g->Finalize(x3, {10, 11, 12});
        Result r3 = g->Search(xb.data(), 128, 10);
        check(r3.size() == 3 && r3[0].first == 10, "k_greater_than_ntotal");
    }
    std::printf("DONE failures=%d\n", g_fail);
    return g_fail ? 1 : 0;
}
