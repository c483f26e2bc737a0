#!/usr/bin/env bash
# A/B of IVF scan builds: the in-tree library and every tunelib/*.so (IVF line, no suite / alt forms / C5).
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
run() {
    local name="$1"; shift
    env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-suite --no-alt-forms --no-c5 > gpurun_out/ivf_$name.json 2> gpurun_out/ivf_$name.err || { tail -5 gpurun_out/ivf_$name.err; return 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ivf_$name.json')); r=d['roofline']
print('$name', d['value'], d['ms_per_step'], r['kernel_ms'], r['merge_ms'], r['frac'], d['recall_at_10'], d['ivf']['rerank_fallbacks_total'])"
}
run base HIPANN_X=0 || exit 1
for f in tunelib/*.so; do
    n=$(basename $f .so)
    run $n HIPANN_LIB=$f || exit 1
done
run base2 HIPANN_X=0 || exit 1
