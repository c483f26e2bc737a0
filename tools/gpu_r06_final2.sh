#!/bin/bash
# r06 final-tree evidence after the one-term IVF items: the whole -m gpu suite and smoke, the IVF scan's kernel-trace
# and FETCH_SIZE passes (tools/gpu_r06_prof.sh ivf, whose pmc_<key>.json is copied into profiles/r06/ first so that the
# bench line's traffic describes this kernel), then the default bench line.  A crash ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-r06g}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_suite.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_suite.log
cp gpurun_out/probe_parity.json gpurun_out/${TAG}_probe_parity.json 2>/dev/null
cp gpurun_out/parity_calibration.json gpurun_out/${TAG}_parity_calibration.json 2>/dev/null
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash tools/gpu_r06_prof.sh ${PROF:-ivf} || exit 1
for f in gpurun_out/pmc_*.json; do cp "$f" profiles/r06/; done
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/${TAG}_bench_detail.json
head -c 1500 gpurun_out/${TAG}_bench.json; echo
