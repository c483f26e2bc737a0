// ivf.hpp — IVFFlat entry points shared between hip_ann.cpp and ivf.cpp.
#pragma once
#include "runtime.hpp"

namespace hipann {
void flat_shard_search(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                       int64_t *I, hipStream_t st);
}  // namespace hipann
