#!/usr/bin/env bash
# A/B of DiskANN traversal builds: the in-tree library and every tunelib/*.so, C4 bench line each.
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
run() {
    local name="$1"; shift
    env "$@" timeout -k 10 200 python bench.py --workload diskann --no-cpu-baseline --steps 10 > gpurun_out/bfs_$name.json 2> gpurun_out/bfs_$name.err || { tail -5 gpurun_out/bfs_$name.err; return 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/bfs_$name.json')); r=d['roofline']
print('$name', d['value'], r['kernel_ms_per_batch'], r['frac'], d['recall_at_10'], d.get('ids_equal_to_oracle_bfs'))"
    grep bfs-prof gpurun_out/bfs_$name.err | tail -1 || true
}
run base HIPANN_X=0 || exit 1
for f in tunelib/*.so; do
    n=$(basename $f .so)
    run $n HIPANN_LIB=$f || exit 1
done
