#!/usr/bin/env bash
# A/B the IVF scan kernel on the GPU box: the in-tree library and every tune/libhipann_*.so, same
# bench command, kernel time from the bench's in-library HIP events.
#   tools/ab_ivf.sh [extra bench args...]   → gpurun_out/ab_<name>.json, summary on stdout
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
run() {
    local name="$1" lib="$2"; shift 2
    HIPANN_LIB="$lib" timeout -k 10 240 python3 "$root/bench.py" --no-cpu-baseline --steps 10 --warmup 3 "$@" \
        > "$root/gpurun_out/ab_$name.json" 2> "$root/gpurun_out/ab_$name.err"
    local rc=$?
    echo "$name rc=$rc $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"recall_at_10": [0-9.]*' "$root/gpurun_out/ab_$name.json" | tr '\n' ' ')"
    return $rc
}
run base "$root/duckdb-annsearch_amd/libhipann.so" "$@" || exit 1
for f in "$root"/tune/libhipann_*.so; do
    [ -e "$f" ] || continue
    n=$(basename "$f" .so); n=${n#libhipann_}
    run "$n" "$f" "$@" || exit 1
done
