#!/bin/bash
# r06: (1) the host-sanitized FaissIndex harness and the harness GPU test; (2) the roctx ranges of one headline run
# under rocprofv3 --marker-trace (HIPANN_ROCTX=1); (3) the fp16 IVF scan's item → XCD mapping A/B (tools/gpu_r06_remap.sh).
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_sanitizers.py tests/test_harness_gpu.py -m gpu -v --timeout 600 \
    --timeout-method thread > gpurun_out/r06m_san.log 2>&1 || { tail -30 gpurun_out/r06m_san.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/r06m_san.log | tail -5
(cd /tmp && export TMPDIR=/tmp && HIPANN_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace \
    --output-format csv -d "$root/gpurun_out/r06m_roctx" -o run -- python3 "$root/bench.py" --workload ivf \
    --no-cpu-baseline --no-suite --no-alt-forms --no-c5 --steps 5 --warmup 2 > "$root/gpurun_out/r06m_roctx.log" 2>&1) \
    || { tail -10 gpurun_out/r06m_roctx.log; exit 1; }
python3 tools/roctx_summary.py gpurun_out/r06m_roctx | tee gpurun_out/r06m_roctx_summary.txt
[ -n "$NO_REMAP" ] || bash tools/gpu_r06_remap.sh
