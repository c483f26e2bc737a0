#!/usr/bin/env bash
# The round's GPU evidence in one call: the whole -m gpu suite, then rocprofv3 kernel-trace/stats and a
# separate FETCH_SIZE PMC pass (tools/gpu_profile.sh) for the IVF (default bench), DiskANN and Flat workloads.
#   tools/gpu_round_profiles.sh   → gpurun_out/pytest_gpu.log, gpurun_out/prof_{ivf,diskann,flat}/, gpurun_out/pmc_*.json
set -uo pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_profile.sh ivf ivf_scan_mfma_bf --no-alt-forms || exit 1
bash tools/gpu_profile.sh diskann diskann_bfs || exit 1
bash tools/gpu_profile.sh flat flat_gemm_topk_bf --no-alt-forms || exit 1
ls gpurun_out/prof_ivf/stats gpurun_out/prof_diskann/stats gpurun_out/prof_flat/stats
cat gpurun_out/pmc_ivf.json gpurun_out/pmc_diskann.json gpurun_out/pmc_flat.json
