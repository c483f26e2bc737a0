set -uo pipefail
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1; echo "dist rc=$?"; tail -3 gpurun_out/pytest_dist.log
tools/gpu_bfs_ab.sh
