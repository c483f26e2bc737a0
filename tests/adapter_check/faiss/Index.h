// Test infrastructure: faiss::Index and faiss::SearchParameters as FAISS 1.13.2 declares them (faiss/Index.h),
// restricted to the members the adapter touches plus every pure virtual (the adapter's classes must be
// concrete).  Signatures restated from FAISS's public header; see MetricType.h.
#pragma once
#include <cstddef>
#include <cstdint>

#include "MetricType.h"

namespace faiss {
struct IDSelector;
struct RangeSearchResult;

struct SearchParameters {
    IDSelector *sel = nullptr;
    virtual ~SearchParameters() {}
};

struct Index {
    int d;
    idx_t ntotal;
    bool verbose;
    bool is_trained;
    MetricType metric_type;
    float metric_arg;

    explicit Index(idx_t d = 0, MetricType metric = METRIC_L2);
    virtual ~Index();
    virtual void train(idx_t n, const float *x);
    virtual void add(idx_t n, const float *x) = 0;
    virtual void add_with_ids(idx_t n, const float *x, const idx_t *xids);
    virtual void search(idx_t n, const float *x, idx_t k, float *distances, idx_t *labels,
                        const SearchParameters *params = nullptr) const = 0;
    virtual void range_search(idx_t n, const float *x, float radius, RangeSearchResult *result,
                              const SearchParameters *params = nullptr) const;
    virtual void assign(idx_t n, const float *x, idx_t *labels, idx_t k = 1) const;
    virtual void reset() = 0;
    virtual size_t remove_ids(const IDSelector &sel);
    virtual void reconstruct(idx_t key, float *recons) const;
    virtual void reconstruct_batch(idx_t n, const idx_t *keys, float *recons) const;
    virtual void reconstruct_n(idx_t i0, idx_t ni, float *recons) const;
};
}  // namespace faiss
