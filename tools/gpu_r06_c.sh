#!/bin/bash
# r06c: the whole -m gpu suite, the C3 test on fp32 coarse keys (A/B of the probe-list differences), the σ = 0.3
# mixture probe (parallel fallback), smoke, the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 300 --timeout-method thread \
    > gpurun_out/r06c_gpu_suite.log 2>&1
rc=$?
tail -12 gpurun_out/r06c_gpu_suite.log | cut -c1-400
cp gpurun_out/probe_parity.json gpurun_out/r06c_probe_parity.json 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite ended with $rc"; exit 1; fi
HIPANN_COARSE_BF3=0 timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -q -k "nlist1024 or 2m_rows" \
    --timeout 300 --timeout-method thread > gpurun_out/r06c_fp32keys.log 2>&1
tail -3 gpurun_out/r06c_fp32keys.log; grep -h '"probe_lists_differing"' gpurun_out/probe_parity.json | sort | uniq -c
timeout -k 10 400 python -u tools/ivf_clustered_probe.py 0.3 10000000 1,8 6,5 > gpurun_out/r06c_probe.log 2>&1 || { tail -20 gpurun_out/r06c_probe.log; exit 1; }
cat gpurun_out/r06c_probe.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r06c_smoke.log; exit 1; }
tail -1 gpurun_out/r06c_smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || { echo "bench failed"; tail -30 gpurun_out/r06c_bench.err; exit 1; }
cat gpurun_out/r06c_bench.json
grep "process at exit" gpurun_out/r06c_bench.err
exit $rc
