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
//   GpuToCpu: back to a CPU IndexFlat / IndexIVFFlat                             :62-75
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

struct Handle {
    void *h = nullptr;
    explicit Handle(void *p) : h(p) {}
    ~Handle() { hipann_free(h); }
    Handle(const Handle &) = delete;
    Handle &operator=(const Handle &) = delete;
};

void check(int rc, const char *err) {
    if (rc != 0) throw std::runtime_error(std::string("HIP search failed: ") + err);
}

}  // namespace

// A faiss::Index whose search runs on the MI355X (the HipIndexFlat of SURVEY §8b B1).
class HipIndexFlat : public faiss::Index {
public:
    HipIndexFlat(const faiss::IndexFlat &cpu) : faiss::Index(cpu.d, cpu.metric_type) {
        char err[512] = {0};
        void *h = hipann_flat_create((int)cpu.d, to_hip_metric(cpu.metric_type), cpu.get_xb(), cpu.ntotal, nullptr,
                                     0, err, sizeof err);
        if (!h) throw std::runtime_error(std::string("hipann_flat_create: ") + err);
        handle_ = std::make_unique<Handle>(h);
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

private:
    std::unique_ptr<Handle> handle_;
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
        handle_ = std::make_unique<Handle>(h);
        ntotal = cpu.ntotal;
        is_trained = true;
        nprobe_ = cpu.nprobe;
    }
    void add(faiss::idx_t, const float *) override {
        throw std::runtime_error("HipIndexIVFFlat::add: the GPU copy is invalidated on append (faiss_index.cpp:469)");
    }
    void search(faiss::idx_t n, const float *x, faiss::idx_t k, float *distances, faiss::idx_t *labels,
                const faiss::SearchParameters *params = nullptr) const override {
        if (k <= 0) throw std::runtime_error("k must be > 0");
        // FaissIndex::Search sets nprobe on the CPU index before each search (faiss_index.cpp:720-726);
        // honour IVF search parameters when given.
        if (auto *ip = dynamic_cast<const faiss::SearchParametersIVF *>(params)) {
            if (ip->nprobe > 0) hipann_ivf_set_nprobe(handle_->h, (int)ip->nprobe);
        } else {
            hipann_ivf_set_nprobe(handle_->h, (int)nprobe_);
        }
        char err[512] = {0};
        check(hipann_ivf_search(handle_->h, n, x, k, distances, reinterpret_cast<int64_t *>(labels), err, sizeof err),
              err);
    }
    void reset() override { throw std::runtime_error("HipIndexIVFFlat::reset: rebuild from the CPU index"); }
    void set_nprobe(size_t np) { nprobe_ = np; }

private:
    std::unique_ptr<Handle> handle_;
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
        if (auto *f = dynamic_cast<HipIndexFlat *>(gpu_index)) {
            auto cpu = std::make_unique<faiss::IndexFlat>(f->d, f->metric_type);
            std::vector<float> row(f->d);
            for (faiss::idx_t i = 0; i < f->ntotal; ++i) {
                f->reconstruct(i, row.data());
                cpu->add(1, row.data());
            }
            return cpu;
        }
        throw std::runtime_error("Index is not a HIP Flat index -- keep the CPU index authoritative");
    }
};

GpuBackend &GetGpuBackend() {
    static HipGpuBackend instance;
    return instance;
}

}  // namespace duckdb

#endif  // HIP_ANN_ENABLED
#endif  // FAISS_AVAILABLE
