#!/usr/bin/env bash
# A/B of Flat builds: the in-tree library and every tunelib/*.so (Flat 10M L2 + IP, 1M L2 lines).
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
run() {
    local name="$1"; shift
    for cfg in "10000000 l2" "10000000 ip" "1000000 l2"; do
        set -- $cfg
        env HIPANN_LIB="${LIBF:-}" timeout -k 10 240 python bench.py --workload flat --n $1 --metric $2 --no-cpu-baseline --no-alt-forms --no-suite --steps 5 > gpurun_out/flat_$name.json 2> gpurun_out/flat_$name.err || { tail -5 gpurun_out/flat_$name.err; return 1; }
        python3 -c "
import json; d=json.load(open('gpurun_out/flat_$name.json')); r=d['roofline']
print('$name', '$1', '$2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('rerank_fallbacks_total'))"
    done
}
LIBF= run base || exit 1
for f in tunelib/*.so; do
    n=$(basename $f .so)
    LIBF=$f run $n || exit 1
done
