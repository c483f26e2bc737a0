#!/usr/bin/env bash
# A/B the IVF list-scan forms on the GPU box (same library, HIPANN_IVF_FORM per run).
#   tools/ab_form.sh "0 3 4" [extra bench args...]   → gpurun_out/abf_<form>.json, summary on stdout
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
forms="$1"; shift
mkdir -p "$root/gpurun_out"
for f in $forms; do
    HIPANN_IVF_FORM=$f timeout -k 10 240 python3 "$root/bench.py" --no-cpu-baseline --steps 10 --warmup 3 "$@" \
        > "$root/gpurun_out/abf_$f.json" 2> "$root/gpurun_out/abf_$f.err" || exit 1
    echo "form $f $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"recall_at_10": [0-9.]*' "$root/gpurun_out/abf_$f.json" | tr '\n' ' ')"
done
