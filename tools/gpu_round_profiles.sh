#!/usr/bin/env bash
# The round's GPU evidence in one call: the whole -m gpu suite, the default bench line, then per
# configuration a rocprofv3 kernel-trace/stats pass and a separate FETCH_SIZE PMC pass (tools/gpu_profile.sh)
# for IVF 10M (default bench), Flat 10M and 1M (L2), and DiskANN C4.
#   tools/gpu_round_profiles.sh            → gpurun_out/pytest_gpu.log, gpurun_out/bench_default.json
#   tools/gpu_round_profiles.sh --no-tests → the profiles only:
#                                               gpurun_out/prof_<key>/, gpurun_out/pmc_<key>.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
if [ "${1:-}" != "--no-tests" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
    tail -1 gpurun_out/pytest_gpu.log
fi
if [ "${1:-}" != "--no-tests" ]; then
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
    || { tail -20 gpurun_out/bench_default.err; exit 1; }
exit 0
fi
bash tools/gpu_profile.sh ivf ivf_scan_mfma_h ivf_10000000x768 --no-alt-forms --no-c5 --steps 10 || exit 1
# Flat form 4: the seed keys pass + passes A and B of flat_bf16_k64 per step (PER_STEP=3: their sum)
PER_STEP=3 bash tools/gpu_profile.sh flat flat_bf16_k64 flat_10000000x768 --no-alt-forms --no-c5 --steps 5 || exit 1
PER_STEP=3 bash tools/gpu_profile.sh flat flat_bf16_k64 flat_1000000x768 --no-alt-forms --no-c5 --n 1000000 --steps 10 || exit 1
bash tools/gpu_profile.sh diskann diskann_bfs diskann_1000000x1536 --steps 10 || exit 1
PER_STEP=3 bash tools/gpu_profile.sh flat flat_bf16_k64 flat_12500000x768_ip --no-alt-forms --no-c5 --n 12500000 --metric ip --steps 5 || exit 1
for key in ivf_10000000x768 flat_10000000x768 flat_1000000x768 diskann_1000000x1536 flat_12500000x768_ip; do
    echo "== $key"; cat gpurun_out/pmc_$key.json
done
