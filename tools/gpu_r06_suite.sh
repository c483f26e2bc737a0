#!/bin/bash
# r06: the -m gpu suite (up to 10 failures reported), smoke, an optional extra step, then the default bench line.
# Each GPU step under its own time limit; a crash / time limit ends the script.
#   tools/gpu_r06_suite.sh TAG ["extra command"]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r06}
EXTRA=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_suite.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_gpu_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite ended with $rc"; exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ -n "$EXTRA" ]; then
    timeout -k 10 900 bash -c "$EXTRA" > gpurun_out/${TAG}_extra.log 2>&1 || { echo "extra failed"; tail -30 gpurun_out/${TAG}_extra.log; exit 1; }
    tail -12 gpurun_out/${TAG}_extra.log
fi
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
exit $rc
