#!/bin/bash
# r03: DiskANN speculative next-row fetch — GPU tests of the traversal, A/B of the C4 line against a
# build without the speculation (HIPANN_BFS_SPEC=0), the per-phase profile of both (HIPANN_BFS_PROF=1),
# then (FULL=1) the whole -m gpu suite, smoke and the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_diskann_gpu.py tests/test_configs_gpu.py -m gpu -k "diskann or c4 or bfs or resident" \
  > gpurun_out/bfs_tests.log 2>&1 || { echo "bfs tests failed"; tail -50 gpurun_out/bfs_tests.log; exit 1; }
tail -2 gpurun_out/bfs_tests.log
B="python3 bench.py --workload diskann --no-cpu-baseline --no-suite --no-c5 --steps 10 --warmup 2"
for rep in 1 2; do
  for lib in "" tunelib/libhipann_nospec.so; do
    HIPANN_LIB=$lib timeout -k 10 300 $B > gpurun_out/bfs_ab.json 2> gpurun_out/bfs_ab.err \
      || { echo "bench failed ($lib)"; tail -20 gpurun_out/bfs_ab.err; exit 1; }
    python3 - "${lib:-spec}" <<'PY'
import json, sys
for l in open('gpurun_out/bfs_ab.json'):
    if l.startswith('{'):
        j = json.loads(l); r = j['roofline']
        print(f"{sys.argv[1]:32s} {j['value']:9.1f} QPS  step {j['ms_per_step']:.3f} ms  kernel {r.get('kernel_ms')} ms  frac {r['frac']:.3f}  recall {j.get('recall_at_10')}")
PY
  done
done
for lib in tunelib/libhipann_prof.so tunelib/libhipann_prof0.so; do
  HIPANN_LIB=$lib timeout -k 10 300 $B --steps 2 > /dev/null 2> gpurun_out/bfs_prof.err || { echo "prof failed"; tail -20 gpurun_out/bfs_prof.err; exit 1; }
  echo "$lib: $(grep bfs-prof gpurun_out/bfs_prof.err | tail -1)"
done
[ "${FULL:-0}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_suite.log 2>&1 || { echo "suite failed"; tail -60 gpurun_out/r03_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r03_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo "bench failed"; tail -30 gpurun_out/r03_bench.err; exit 1; }
echo bench ok
bash tools/gpu_ivf_trace.sh || { echo "ivf trace failed"; exit 1; }
python3 tools/trace_summary.py gpurun_out/trace_ivf_nq1024 > gpurun_out/ivf_step_breakdown.txt && cat gpurun_out/ivf_step_breakdown.txt
python3 tools/trace_summary.py gpurun_out/trace_ivf_nq1 > gpurun_out/ivf_step_breakdown_nq1.txt && cat gpurun_out/ivf_step_breakdown_nq1.txt
