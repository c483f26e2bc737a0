#!/bin/bash
# r04: the IVF rerank's per-phase clocks (tuning build libhipann_rrprof.so, HIPANN_RR_PROF=1) on the default line.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
HIPANN_LIB=$(pwd)/duckdb-annsearch_amd/libhipann_rrprof.so HIPANN_RR_PROF_DUMP=1 timeout -k 10 300 python -u bench.py \
    --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 3 > gpurun_out/rrprof.json 2> gpurun_out/rrprof.err \
    || { echo "rrprof failed"; tail -20 gpurun_out/rrprof.err; exit 1; }
grep "rerank phase" gpurun_out/rrprof.err
