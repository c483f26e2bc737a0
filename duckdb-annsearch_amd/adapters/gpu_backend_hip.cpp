// gpu_backend_hip.cpp — the extension's GpuBackend implemented on the MI355X C ABI (hip_ann.h).
//
// Drop-in replacement of src/gpu_backend_metal.mm (MetalGpuBackend, :14-84) for a DuckDB `ann`
// build with -DHIP_ANN_ENABLED (the analogue of FAISS_METAL_ENABLED, CMakeLists.txt:142-174,
// :271-303).  Compiled only where FAISS and the extension headers exist (FAISS_AVAILABLE); in this
// repository it is built by no target (FAISS is not installed) — INTEGRATION.md shows the CMake lines.
//
// Behaviour mirrored:
//   IsAvailable / DeviceInfo / BackendName     gpu_backend_metal.mm:33-45
//   CpuToGpu: IndexIVFFlat first, then IndexFlat, else throw std::runtime_error   :45-60
//   GpuToCpu: back to a CPU IndexIVFFlat / IndexFlat                             :62-75
//             (index_metal_to_cpu_ivf, MetalIndexIVFFlat.mm:328-356: flat quantizer over the centroids,
//             own_fields, is_trained, nprobe, invlists->add_entries per list, ntotal)
//   search(): MetalIndexFlat::search contract (MetalIndexFlat.mm:294-369): k <= 0 throws,
//             effective_k = min(k, ntotal), (+inf | -inf, -1) pads, int64 labels.
//   Errors are std::runtime_error (faiss_index.cpp:122-124, :146-148 catch exactly that type).
#ifdef FAISS_AVAILABLE
#ifdef HIP_ANN_ENABLED

#include "gpu_backend.hpp"
#include "hip_ann.h"

#include <faiss/IndexFlat.h>
#include <faiss/IndexIVFFlat.h>
#include <faiss/invlists/InvertedLists.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace duckdb {

namespace {

int to_hip_metric(faiss::MetricType m) {
    if (m == faiss::METRIC_L2) return HIPANN_METRIC_L2;
    if (m == faiss::METRIC_INNER_PRODUCT) return HIPANN_METRIC_IP;
    throw std::runtime_error("HIP GPU backend supports METRIC_L2 and METRIC_INNER_PRODUCT only");
}

void check(int rc, const char *err) {
    if (rc != 0) throw std::runtime_error(std::string("HIP search failed: ") + err);
}

}  // namespace

// Owner of a libhipann handle (hipann_free on destruction).  A named type: the index classes below have external
// linkage, so their members must not use the anonymous namespace.
struct HipAnnHandle {
    void *h = nullptr;
    explicit HipAnnHandle(void *p) : h(p) {}
    ~HipAnnHandle() { hipann_free(h); }
    HipAnnHandle(const HipAnnHandle &) = delete;
    HipAnnHandle &operator=(const HipAnnHandle &) = delete;
};

// A faiss::Index whose search runs on the MI355X (the HipIndexFlat of SURVEY §8b B1).
class HipIndexFlat : public faiss::Index {
public:
    HipIndexFlat(const faiss::IndexFlat &cpu) : faiss::Index(cpu.d, cpu.metric_type) {
        char err[512] = {0};
        void *h = hipann_flat_create((int)cpu.d, to_hip_metric(cpu.metric_type), cpu.get_xb(), cpu.ntotal, nullptr,
                                     0, err, sizeof err);
        if (!h) throw std::runtime_error(std::string("hipann_flat_create: ") + err);
        handle_ = std::make_unique<HipAnnHandle>(h);
        ntotal = cpu.ntotal;
        is_trained = true;
    }
    void add(faiss::idx_t n, const float *x) override {
        char err[512] = {0};
        check(hipann_flat_add(handle_->h, x, n, err, sizeof err), err);
        ntotal += n;
    }
    void search(faiss::idx_t n, const float *x, faiss::idx_t k, float *distances, faiss::idx_t *labels,
                const faiss::SearchParameters * = nullptr) const override {
        if (k <= 0) throw std::runtime_error("k must be > 0");
        char err[512] = {0};
        check(hipann_flat_search(handle_->h, n, x, k, distances, reinterpret_cast<int64_t *>(labels), err, sizeof err),
              err);
    }
    void reset() override { throw std::runtime_error("HipIndexFlat::reset: rebuild from the CPU index"); }
    void reconstruct(faiss::idx_t key, float *recons) const override {
        char err[512] = {0};
        check(hipann_flat_reconstruct(handle_->h, key, recons, err, sizeof err), err);
    }
    void *handle() const { return handle_->h; }

private:
    std::unique_ptr<HipAnnHandle> handle_;
};

class HipIndexIVFFlat : public faiss::Index {
public:
    HipIndexIVFFlat(const faiss::IndexIVFFlat &cpu) : faiss::Index(cpu.d, cpu.metric_type), nlist_(cpu.nlist) {
        auto *flatq = dynamic_cast<const faiss::IndexFlat *>(cpu.quantizer);
        if (!flatq) throw std::runtime_error("HIP IVFFlat needs a flat coarse quantizer");
        std::vector<int64_t> offsets(cpu.nlist + 1, 0);
        for (size_t l = 0; l < cpu.nlist; ++l) offsets[l + 1] = offsets[l] + (int64_t)cpu.invlists->list_size(l);
        std::vector<int64_t> ids((size_t)offsets[cpu.nlist]);
        std::vector<float> codes((size_t)offsets[cpu.nlist] * cpu.d);
        for (size_t l = 0; l < cpu.nlist; ++l) {  // ArrayInvertedLists → CSR (codes are raw fp32 rows)
            const size_t sz = cpu.invlists->list_size(l);
            if (!sz) continue;
            faiss::InvertedLists::ScopedIds li(cpu.invlists, l);
            faiss::InvertedLists::ScopedCodes lc(cpu.invlists, l);
            std::copy(li.get(), li.get() + sz, ids.begin() + offsets[l]);
            std::memcpy(codes.data() + offsets[l] * cpu.d, lc.get(), sz * cpu.d * sizeof(float));
        }
        char err[512] = {0};
        void *h = hipann_ivf_create((int)cpu.d, to_hip_metric(cpu.metric_type), (int)cpu.nlist, (int)cpu.nprobe,
                                    flatq->get_xb(), offsets.data(), ids.data(), codes.data(), nullptr, 0, err,
                                    sizeof err);
        if (!h) throw std::runtime_error(std::string("hipann_ivf_create: ") + err);
        handle_ = std::make_unique<HipAnnHandle>(h);
        ntotal = cpu.ntotal;
        is_trained = true;
        nprobe_ = cpu.nprobe;
    }
    // IndexIVF::add / add_with_ids on the GPU copy: hipann_ivf_add assigns the rows with the GPU coarse
    // quantizer and appends them to their lists (labels ntotal + i, or xids).
    void add(faiss::idx_t n, const float *x) override { add_with_ids(n, x, nullptr); }
    void add_with_ids(faiss::idx_t n, const float *x, const faiss::idx_t *xids) override {
        char err[512] = {0};
        check(hipann_ivf_add(handle_->h, n, x, reinterpret_cast<const int64_t *>(xids), err, sizeof err), err);
        ntotal += n;
    }
    void search(faiss::idx_t n, const float *x, faiss::idx_t k, float *distances, faiss::idx_t *labels,
                const faiss::SearchParameters *params = nullptr) const override {
        if (k <= 0) throw std::runtime_error("k must be > 0");
        // FaissIndex::Search sets nprobe on the CPU index before each search (faiss_index.cpp:720-726);
        // IVF search parameters override it per call.  The value travels with the call and is read under
        // the handle's lock (hipann_ivf_search_np), so concurrent searches with different nprobe are safe.
        int np = (int)nprobe_;
        if (auto *ip = dynamic_cast<const faiss::SearchParametersIVF *>(params))
            if (ip->nprobe > 0) np = (int)ip->nprobe;
        char err[512] = {0};
        check(hipann_ivf_search_np(handle_->h, np, n, x, k, distances, reinterpret_cast<int64_t *>(labels), err,
                                   sizeof err),
              err);
    }
    void reset() override { throw std::runtime_error("HipIndexIVFFlat::reset: rebuild from the CPU index"); }
    void set_nprobe(size_t np) { nprobe_ = np; }
    size_t nprobe() const { return nprobe_; }
    size_t nlist() const { return nlist_; }
    void *handle() const { return handle_->h; }

private:
    std::unique_ptr<HipAnnHandle> handle_;
    size_t nlist_ = 0, nprobe_ = 1;
};

class HipGpuBackend : public GpuBackend {
public:
    bool IsAvailable() const override { return hipann_available() == 1; }
    std::string DeviceInfo() const override {
        if (!IsAvailable()) return "HIP: not available";
        char buf[512] = {0};
        hipann_device_info(buf, sizeof buf);
        return std::string("HIP GPU (") + buf + ")";
    }
    std::string BackendName() const override { return "hip"; }
    std::unique_ptr<faiss::Index> CpuToGpu(faiss::Index *cpu_index) override {
        if (!IsAvailable()) throw std::runtime_error("HIP GPU backend not available");
        if (auto *ivf = dynamic_cast<faiss::IndexIVFFlat *>(cpu_index)) return std::make_unique<HipIndexIVFFlat>(*ivf);
        if (auto *flat = dynamic_cast<faiss::IndexFlat *>(cpu_index)) return std::make_unique<HipIndexFlat>(*flat);
        throw std::runtime_error("HIP GPU supports IndexFlat and IndexIVFFlat. Got an unsupported index type.");
    }
    std::unique_ptr<faiss::Index> GpuToCpu(faiss::Index *gpu_index) override {
        if (auto *v = dynamic_cast<HipIndexIVFFlat *>(gpu_index)) {
            // index_metal_to_cpu_ivf (MetalIndexIVFFlat.mm:328-356) from the HBM lists
            const int nlist = (int)v->nlist(), d = (int)v->d;
            char err[512] = {0};
            std::vector<int64_t> off(nlist + 1);
            check(hipann_ivf_export(v->handle(), nullptr, off.data(), nullptr, nullptr, err, sizeof err), err);
            std::vector<float> cen((size_t)nlist * d), codes((size_t)off[nlist] * d);
            std::vector<int64_t> ids((size_t)off[nlist]);
            check(hipann_ivf_export(v->handle(), cen.data(), off.data(), ids.data(), codes.data(), err, sizeof err), err);
            auto *quantizer = new faiss::IndexFlat(d, v->metric_type);
            quantizer->add(nlist, cen.data());
            auto cpu = std::make_unique<faiss::IndexIVFFlat>(quantizer, d, nlist, v->metric_type);
            cpu->own_fields = true;
            cpu->is_trained = true;
            cpu->nprobe = v->nprobe();
            for (int l = 0; l < nlist; ++l) {
                const size_t len = (size_t)(off[l + 1] - off[l]);
                if (!len) continue;
                cpu->invlists->add_entries(l, len, reinterpret_cast<const faiss::idx_t *>(ids.data() + off[l]),
                                           reinterpret_cast<const uint8_t *>(codes.data() + (size_t)off[l] * d));
            }
            cpu->ntotal = off[nlist];
            return cpu;
        }
        if (auto *f = dynamic_cast<HipIndexFlat *>(gpu_index)) {  // index_metal_to_cpu
            auto cpu = std::make_unique<faiss::IndexFlat>(f->d, f->metric_type);
            std::vector<float> xb((size_t)f->ntotal * f->d);
            char err[512] = {0};
            check(hipann_flat_reconstruct_n(f->handle(), 0, f->ntotal, xb.data(), err, sizeof err), err);
            cpu->add(f->ntotal, xb.data());
            return cpu;
        }
        throw std::runtime_error("Index is not a HIP index -- cannot convert to CPU");
    }
};

GpuBackend &GetGpuBackend() {
    static HipGpuBackend instance;
    return instance;
}

}  // namespace duckdb

#endif  // HIP_ANN_ENABLED
#endif  // FAISS_AVAILABLE
