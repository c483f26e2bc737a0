// Test infrastructure: faiss::Level1Quantizer / IndexIVFInterface / IndexIVF / SearchParametersIVF (FAISS 1.13.2
// faiss/IndexIVF.h), the members the adapter uses: quantizer, nlist, own_fields, nprobe, invlists, the
// SearchParametersIVF::nprobe override.  See MetricType.h.
#pragma once
#include <cstddef>

#include "Index.h"
#include "invlists/InvertedLists.h"

namespace faiss {
struct Level1Quantizer {
    Index *quantizer = nullptr;
    size_t nlist = 0;
    char quantizer_trains_alone = 0;
    bool own_fields = false;
    Level1Quantizer(Index *quantizer, size_t nlist);
    Level1Quantizer();
    ~Level1Quantizer();
};

struct SearchParametersIVF : SearchParameters {
    size_t nprobe = 1;
    size_t max_codes = 0;
    SearchParameters *quantizer_params = nullptr;
    void *inverted_list_context = nullptr;
    ~SearchParametersIVF() {}
};

struct IndexIVFInterface : Level1Quantizer {
    size_t nprobe = 1;
    size_t max_codes = 0;
    explicit IndexIVFInterface(Index *quantizer = nullptr, size_t nlist = 0);
    virtual ~IndexIVFInterface() {}
};

struct IndexIVF : Index, IndexIVFInterface {
    InvertedLists *invlists = nullptr;
    bool own_invlists = false;
    size_t code_size = 0;
    IndexIVF(Index *quantizer, size_t d, size_t nlist, size_t code_size, MetricType metric = METRIC_L2,
             bool own_invlists = true);
    IndexIVF();
    void reset() override;
    void train(idx_t n, const float *x) override;
    void add(idx_t n, const float *x) override;
    void add_with_ids(idx_t n, const float *x, const idx_t *xids) override;
    void search(idx_t n, const float *x, idx_t k, float *distances, idx_t *labels,
                const SearchParameters *params = nullptr) const override;
    void reconstruct(idx_t key, float *recons) const override;
    ~IndexIVF() override;
};
}  // namespace faiss
