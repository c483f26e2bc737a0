// ivf.hpp — internal entry points shared between the C ABI translation units.
#pragma once
#include "runtime.hpp"

namespace hipann {
// form_override >= 0 replaces ix.form for this call (the exact forms' re-run of flagged queries).  pend == nullptr:
// the whole search (one host synchronisation when an exact form's flag count must be read); otherwise only the
// launch phase — no host synchronisation — and *pend holds what flat_shard_finish must run after the caller has
// synchronised with `st` (hipann_flat_search: every shard launched before any is waited on).
void flat_shard_search(FlatIndex &ix, FlatShard &sh, int64_t nq, const float *xq, int k, int kout, float *D,
                       int64_t *I, hipStream_t st, int form_override = -1, FlatPending *pend = nullptr);
void flat_shard_finish(FlatIndex &ix, FlatShard &sh, const FlatPending &pend, hipStream_t st);
// form_override >= 0 replaces ix.form for this call (the exact form's re-run of flagged queries)
// probes_in (device, nq × min(nprobe, nlist) int64): the caller's probe lists replace the coarse quantizer's
void ivf_shard_search(IvfIndex &ix, IvfShard &sh, int64_t nq, const float *xq, int k, int kout, float *D, int64_t *I,
                      hipStream_t st, int form_override = -1, const int64_t *probes_in = nullptr);
}  // namespace hipann
