#!/usr/bin/env bash
set -uo pipefail
root="${GRAFT_REPO_ROOT:-.}"
cd "$root"
tools/gpu_kernel_pmc.sh flat10m flat_bf16_topk --workload flat || exit 1
tools/gpu_kernel_pmc.sh ivf10m ivf_scan_mfma_h --no-c5 || exit 1
tools/gpu_kernel_pmc.sh diskann1m diskann_bfs --workload diskann || exit 1
