#!/bin/bash
# r04: IVF chunk rows A/B (2048 default vs the HIPANN_IVF_CH=4096 tuning build): step time, scan and rerank time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in 2048 4096 2048 4096; do
  if [ $v = 4096 ]; then export HIPANN_LIB=$(pwd)/duckdb-annsearch_amd/libhipann_ch4096.so; else unset HIPANN_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --steps 20 --warmup 3 \
      > gpurun_out/chab_$v.json 2> gpurun_out/chab_$v.err || { echo "chab $v failed"; tail -20 gpurun_out/chab_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/chab_$v.json').read()); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel_ms'], r['merge_ms'], d['recall_at_10'])"
done
