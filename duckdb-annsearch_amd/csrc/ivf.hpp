// ivf.hpp — internal entry points shared between the C ABI translation units.
#pragma once
#include "runtime.hpp"

namespace hipann {
void flat_shard_search(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                       int64_t *I, hipStream_t st);
void ivf_shard_search(IvfIndex &ix, IvfShard &sh, int64_t nq, const float *xq, int k, int kout, float *D, int64_t *I,
                      hipStream_t st);
}  // namespace hipann
