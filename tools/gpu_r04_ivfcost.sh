#!/bin/bash
# r04: IVF 10M x 768 nq 1024 per-step kernel trace (time outside the scan) + SQ counters of the rerank kernel.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/ivfc_breakdown_r04.txt
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
# variants: name=ENV=value (or name= for the default build settings), from $IVFC_VARIANTS
for spec in ${IVFC_VARIANTS:-default= nohook=HIPANN_IVF_SELECT_HOOK=0}; do
  v=${spec%%=*}; envset=${spec#*=}
  unset HIPANN_IVF_SELECT_HOOK HIPANN_ROWSEL_BLOCK HIPANN_KEYS
  if [ -n "$envset" ]; then export "$envset"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/gpurun_out/trace_ivfc_r04_$v" -o run -- \
      python3 "$root/bench.py" --no-cpu-baseline --no-alt-forms --no-suite --no-c5 --nq 1024 --steps 30 --warmup 3 \
      > "$root/gpurun_out/trace_ivfc_r04_$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "$root/gpurun_out/trace_ivfc_r04_$v.log"; exit 1; }
  echo "## $v" >> "$root/gpurun_out/ivfc_breakdown_r04.txt"
  python3 "$root/tools/trace_summary.py" "$root/gpurun_out/trace_ivfc_r04_$v" ivf_scan_mfma_h 8 >> "$root/gpurun_out/ivfc_breakdown_r04.txt"
done
unset HIPANN_IVF_SELECT_HOOK HIPANN_ROWSEL_BLOCK HIPANN_KEYS
cat "$root/gpurun_out/ivfc_breakdown_r04.txt"
if [ -z "$IVFC_PMC" ]; then exit 0; fi
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM \
    SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "ivf_rerank_topk|rows_select_block|ivf_planfill_q|flat_keys_ksplit" \
    --output-format csv -d "$root/gpurun_out/pmc_r04_rr" -o run -- python3 "$root/bench.py" --no-cpu-baseline \
    --no-alt-forms --no-suite --no-c5 --steps 2 --warmup 1 > "$root/gpurun_out/pmc_r04_rr.log" 2>&1 \
    || { echo "pmc failed"; tail -5 "$root/gpurun_out/pmc_r04_rr.log"; exit 1; }
for k in ivf_rerank_topk rows_select_block ivf_planfill_q flat_keys_ksplit; do
  python3 "$root/tools/pmc_summary.py" $k "$root/gpurun_out/pmc_r04_rr" | sed "s#^#$k #"
done | tee "$root/gpurun_out/pmc_r04_rr_summary.txt"
