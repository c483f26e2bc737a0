#!/bin/bash
# r04: C2 (Flat L2 1M x 768, nq 1024) per-step kernel breakdown (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "$(dirname "$0")/.."
root=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for spec in ${C2_VARIANTS:-default=}; do
v=${spec%%=*}; envset=${spec#*=}
unset HIPANN_FLAT_SAMPLE HIPANN_FLAT_CAND_REGS HIPANN_FLAT_KTH_NARROW HIPANN_FLAT_CAND_NARROW HIPANN_FLAT_PASS_A
if [ -n "$envset" ]; then export "$envset"; fi
echo "## $v"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/trace_c2_r04_$v" -o run -- \
    python3 "$root/bench.py" --workload flat --n 1000000 --no-cpu-baseline --no-alt-forms --steps 20 --warmup 3 \
    > "$root/gpurun_out/trace_c2_r04_$v.log" 2>&1 || { echo "trace failed"; tail -5 "$root/gpurun_out/trace_c2_r04_$v.log"; exit 1; }
grep -o '"value": [0-9.]*, "unit": "queries/s", "n_gpus": 1, "steps": 20, "warmup": 3, "ms_per_step": [0-9.]*' "$root/gpurun_out/trace_c2_r04_$v.log" | head -1
python3 - "$root/gpurun_out/trace_c2_r04_$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-60:]
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000; cnt[n] += 1
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:16]:
    print(f"{t / max(cnt[n],1):10.1f} us avg  x{cnt[n]:4d}  {n}")
PY
done
