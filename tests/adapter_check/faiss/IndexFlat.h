// Test infrastructure: faiss::IndexFlatCodes / IndexFlat (FAISS 1.13.2 faiss/IndexFlatCodes.h, faiss/IndexFlat.h),
// the members the adapter uses: the constructor, add (inherited override) and get_xb.  See MetricType.h.
#pragma once
#include <cstdint>
#include <vector>

#include "Index.h"

namespace faiss {
struct IndexFlatCodes : Index {
    size_t code_size;
    std::vector<uint8_t> codes;
    IndexFlatCodes();
    IndexFlatCodes(size_t code_size, idx_t d, MetricType metric = METRIC_L2);
    void add(idx_t n, const float *x) override;
    void reset() override;
};

struct IndexFlat : IndexFlatCodes {
    explicit IndexFlat(idx_t d, MetricType metric = METRIC_L2);
    IndexFlat();
    void search(idx_t n, const float *x, idx_t k, float *distances, idx_t *labels,
                const SearchParameters *params = nullptr) const override;
    void reconstruct(idx_t key, float *recons) const override;
    float *get_xb();
    const float *get_xb() const;
};
}  // namespace faiss
