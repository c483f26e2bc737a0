#!/bin/bash
# r05: the -m gpu suite, smoke, then the default bench line.  Each GPU step under its own time limit; the first
# failure ends the script.  Usage: tools/gpu_r05_suite.sh TAG [pytest selection...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r05}
shift || true
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || { echo "suite failed"; tail -80 gpurun_out/${TAG}_gpu_suite.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
