#!/bin/bash
# r06 roofline evidence: per configuration a rocprofv3 --kernel-trace --stats pass and a separate
# FETCH_SIZE pass (MI355X_MICROARCH.md §HBM: counters in their own run, no trace domains beside --pmc) of the kernel
# the bench line's roofline names, from this tree on one box; pmc_<key>.json per launch (= per search) for bench.py.
#   tools/gpu_r06_prof.sh [config ...]     configs: ivf flat10m c2 c5 diskann (default: all)
# → gpurun_out/r06prof_<cfg>/{stats,pmc}/, gpurun_out/r06prof_<cfg>_{stats,pmc}.log, gpurun_out/pmc_<key>.json
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$root/gpurun_out"
cd /tmp && export TMPDIR=/tmp
o="$root/gpurun_out"
one() {  # cfg key kernel-substring json-kernel-name group-start bench-args...
    local cfg="$1" key="$2" kern="$3" name="$4" grp="$5"; shift 5
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/r06prof_$cfg/stats" -o run -- \
        python3 "$root/bench.py" --no-cpu-baseline --no-suite --no-alt-forms --no-c5 --steps 10 --warmup 3 "$@" \
        > "$o/r06prof_${cfg}_stats.log" 2>&1 || { echo "stats $cfg failed"; tail -5 "$o/r06prof_${cfg}_stats.log"; return 1; }
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$kern" --output-format csv \
        -d "$o/r06prof_$cfg/pmc" -o run -- \
        python3 "$root/bench.py" --no-cpu-baseline --no-suite --no-alt-forms --no-c5 --steps 3 --warmup 1 "$@" \
        > "$o/r06prof_${cfg}_pmc.log" 2>&1 || { echo "pmc $cfg failed"; tail -5 "$o/r06prof_${cfg}_pmc.log"; return 1; }
    if [ -n "$grp" ]; then
        python3 "$root/tools/pmc_traffic.py" "$o/r06prof_$cfg/pmc" "$kern" --skip 2 --group-start "$grp" --name "$name" \
            --out "$o/pmc_$key.json" > /dev/null || return 1
    else
        python3 "$root/tools/pmc_traffic.py" "$o/r06prof_$cfg/pmc" "$kern" --skip 2 --name "$name" \
            --out "$o/pmc_$key.json" > /dev/null || return 1
    fi
    echo "== $cfg: $(grep -h '"ms_per_step"' "$o/r06prof_${cfg}_stats.log" | tail -1 | cut -c1-160)"
    cat "$o/pmc_$key.json"
}
cfgs=${*:-ivf flat10m c2 c5 diskann}
for c in $cfgs; do
    case $c in
        ivf) one ivf ivf_10000000x768 ivf_scan_mfma_h ivf_scan_mfma_h "" --workload ivf || exit 1 ;;
        flat10m) one flat10m flat_10000000x768 flat_bf16_k64 "flat_bf16_k64<I8>" "flat_bf16_k64<true, true" \
                     --workload flat --n 10000000 || exit 1 ;;
        c2) one c2 flat_1000000x768 flat_bf16_k64 "flat_bf16_k64<I8>" "flat_bf16_k64<true, true" \
                --workload flat --n 1000000 || exit 1 ;;
        c5) one c5 flat_12500000x768_ip flat_bf16_k64 "flat_bf16_k64<I8>" "flat_bf16_k64<false, true" \
                --workload flat --n 12500000 --metric ip || exit 1 ;;
        diskann) one diskann diskann_1000000x1536 diskann_bfs diskann_bfs "" --workload diskann --n 1000000 --d 1536 \
                     || exit 1 ;;
        append) PROBE_N=10000000 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
                    -d "$o/r06prof_append/stats" -o run -- python3 "$root/tools/append_probe.py" \
                    > "$o/r06prof_append.log" 2>&1 || { echo "append trace failed"; tail -5 "$o/r06prof_append.log"; exit 1; }
                tail -2 "$o/r06prof_append.log" ;;
    esac
done
