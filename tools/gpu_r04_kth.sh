#!/bin/bash
# r04: the narrowed seed k-th (flat_keys_kth) and candidate bound / select — parity tests, then the C2 / 10M Flat kernel traces (narrowed vs
# HIPANN_FLAT_KTH_NARROW=0) and the IVF step trace with fence-free timing events.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flat_kth_gpu.py tests/test_flat_gpu.py tests/test_request_k_gpu.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
    > gpurun_out/r04_kth_tests.log 2>&1 || { tail -30 gpurun_out/r04_kth_tests.log; exit 1; }
tail -1 gpurun_out/r04_kth_tests.log
C2_VARIANTS="narrow= oldkth=HIPANN_FLAT_KTH_NARROW=0 oldcand=HIPANN_FLAT_CAND_NARROW=0" bash tools/gpu_r04_c2trace.sh || exit 1
IVFC_VARIANTS="evf=" bash tools/gpu_r04_ivfcost.sh || exit 1
