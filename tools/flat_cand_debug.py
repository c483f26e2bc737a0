import sys, numpy as np
sys.path.insert(0, 'duckdb-annsearch_amd')
import torch, hipann
rng = np.random.default_rng(11)
n, d, nq = 1_000_000, int(sys.argv[1]), 512
xb = rng.standard_normal((n, d), dtype=np.float32)
xq = rng.standard_normal((nq, d), dtype=np.float32)
for metric in (0, 1):
    ix = hipann.HipIndexFlat(d, metric, xb)
    ix.form = ix.FORM_FP32
    D0, I0 = ix.search(xq, 10)
    ix.form = ix.FORM_BF16_EXACT
    try:
        D1, I1 = ix.search(xq, 10)
        print(metric, 'match', (I1 == I0).mean(), 'fallbacks', ix.rerank_fallbacks(), flush=True)
    except Exception as e:
        print(metric, 'ERR', e, flush=True)
