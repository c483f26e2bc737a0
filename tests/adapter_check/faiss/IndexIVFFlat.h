// Test infrastructure: faiss::IndexIVFFlat (FAISS 1.13.2 faiss/IndexIVFFlat.h): its constructor.  See MetricType.h.
#pragma once
#include "IndexIVF.h"

namespace faiss {
struct IndexIVFFlat : IndexIVF {
    IndexIVFFlat(Index *quantizer, size_t d, size_t nlist_, MetricType = METRIC_L2, bool own_invlists = true);
    IndexIVFFlat();
};
}  // namespace faiss
