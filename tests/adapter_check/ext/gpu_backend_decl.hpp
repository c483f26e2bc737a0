// Test infrastructure: the extension's GpuBackend interface (reference src/include/gpu_backend.hpp:12-33) as the
// adapter implements it — five pure virtuals and the link-time singleton, under FAISS_AVAILABLE like the
// original.  Declarations only.
#pragma once
#ifdef FAISS_AVAILABLE
#include <faiss/Index.h>

#include <memory>
#include <string>

namespace duckdb {
class GpuBackend {
public:
    virtual ~GpuBackend() = default;
    virtual bool IsAvailable() const = 0;
    virtual std::string DeviceInfo() const = 0;
    virtual std::string BackendName() const = 0;
    virtual std::unique_ptr<faiss::Index> CpuToGpu(faiss::Index *cpu_index) = 0;
    virtual std::unique_ptr<faiss::Index> GpuToCpu(faiss::Index *gpu_index) = 0;
};
GpuBackend &GetGpuBackend();
}  // namespace duckdb
#endif
