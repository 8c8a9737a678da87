#!/bin/bash
# One parameterised GPU-box session (run through gpurun from the repo root):
#   tools/gpu_session.sh <tag> <step> [<step> ...]
# Steps (each under its own time limit; a fault, abort or timeout ends the script):
#   tests            pytest -m gpu (verbose log)
#   ptest:<file>     pytest -m gpu of one test file
#   smoke            __graft_entry__.smoke()
#   bench[:cfg[:args]]   bench.py --config cfg (args: extra bench flags, '+' for spaces)
#   stats[:cfg[:args]]   rocprofv3 --kernel-trace --stats of the same bench
#   pmc[:cfg[:args]]     PMC passes (SQ x2, FETCH_SIZE, WRITE_SIZE), one rocprofv3 run each
#   py:<file>        python3 <file> (ad-hoc probe script)
# Output: gpurun_out/<tag>/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "[$(date +%T)] $name: $*" >> "$OUT/steps.txt"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.txt"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in "$@"; do
    kind=${s%%:*}; rest=${s#*:}; [ "$rest" = "$s" ] && rest=""
    cfg=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
    args=${args//+/ }; cfg=${cfg:-c2}
    case $kind in
        tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 ;;
        ptest) step "ptest_$(basename "$cfg" .py)" 600 python -u -m pytest "$cfg" -m gpu -x -v --timeout 120 --timeout-method thread ;;
        smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) tag=$(echo "$args" | tr -cd 'a-z0-9'); step "bench_${cfg}${tag:+_$tag}" 900 python3 -u bench.py --config "$cfg" $args ;;
        stats) step "stats_${cfg}" 900 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --cpu-baseline 0 $args ;;
        pmc)
            step "pmc_sq1_${cfg}" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d "$OUT/sq1_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --cpu-baseline 0 $args
            step "pmc_sq2_${cfg}" 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$OUT/sq2_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --cpu-baseline 0 $args
            step "pmc_fetch_${cfg}" 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --cpu-baseline 0 $args
            step "pmc_write_${cfg}" 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --cpu-baseline 0 $args
            # per-kernel summary; the raw per-dispatch CSVs of a sweep exceed gpurun's 64 MiB copy-back
            python3 tools/pmc_summary.py "$OUT" "_$cfg" > "$OUT/pmc_summary_$cfg.json"
            rm -rf "$OUT/sq1_$cfg" "$OUT/sq2_$cfg" "$OUT/fetch_$cfg" "$OUT/write_$cfg" ;;
        py) step "py_$(basename "$cfg" .py)" 600 python3 -u "$cfg" $args ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo done >> "$OUT/steps.txt"
