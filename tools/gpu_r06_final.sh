#!/bin/bash
# r06 final-tree evidence: the whole -m gpu suite, smoke, the default bench line, then the r06 profiles of every
# configuration (tools/gpu_r06_prof.sh).  Each GPU step under its own limit; a crash ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r06f}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_suite.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_suite.log
cp gpurun_out/probe_parity.json gpurun_out/${TAG}_probe_parity.json 2>/dev/null
cp gpurun_out/parity_calibration.json gpurun_out/${TAG}_parity_calibration.json 2>/dev/null
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/${TAG}_bench_detail.json
head -c 1500 gpurun_out/${TAG}_bench.json; echo
if [ "${2:-}" = "prof" ]; then bash tools/gpu_r06_prof.sh ivf flat10m c2 c5 diskann || exit 1; fi
