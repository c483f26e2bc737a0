// ivf.hpp — internal entry points shared between the C ABI translation units.
#pragma once
#include "runtime.hpp"

namespace hipann {
// form_override >= 0 replaces ix.form for this call (the exact forms' re-run of flagged queries)
void flat_shard_search(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                       int64_t *I, hipStream_t st, int form_override = -1);
// form_override >= 0 replaces ix.form for this call (the exact form's re-run of flagged queries)
void ivf_shard_search(IvfIndex &ix, IvfShard &sh, int64_t nq, const float *xq, int k, int kout, float *D, int64_t *I,
                      hipStream_t st, int form_override = -1);
}  // namespace hipann
