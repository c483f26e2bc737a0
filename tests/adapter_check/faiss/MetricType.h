// Test infrastructure (compile check of adapters/gpu_backend_hip.cpp, tests/test_adapter_compile.py): the
// declarations of FAISS 1.13.2's faiss/MetricType.h that the adapter uses, restated from FAISS's public
// headers (FAISS is an external dependency of the extension, vcpkg.json:3 / FIXES.md:3; not vendored in the
// reference and not installed here).  Declarations only — nothing here is linked or run.
#pragma once
#include <cstdint>

namespace faiss {
using idx_t = int64_t;
enum MetricType {
    METRIC_INNER_PRODUCT = 0,
    METRIC_L2 = 1,
    METRIC_L1,
    METRIC_Linf,
    METRIC_Lp,
};
}  // namespace faiss
