#!/bin/bash
# rocprofv3 passes for the C2 bench (run on the GPU box from the repo root).
# Each step has its own time limit; a step that faults, aborts or times out
# ends the script.  A rejected counter name (rc 1) only skips that pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${PROF_OUT:-gpurun_out/prof_r01}
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc" >> "$OUT/steps.txt"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
    return 0
}
CFG=${PROF_CONFIG:-c2}
N=${PROF_REPORTS:-12288}
NP=${PMC_REPORTS:-2048}
SKIP=${PROF_SKIP:-}
step list 120 rocprofv3 -L
[ -z "$SKIP" ] && step bench 600 python3 bench.py --config $CFG --reports $N --steps 3 --warmup 1
step stats 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --config $CFG --reports $N --steps 2 --warmup 1 --cpu-baseline 0
[ -z "$SKIP" ] && step pmc_sq1 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $OUT/sq1 -o run --output-format csv -- python3 bench.py --config $CFG --reports $NP --steps 1 --warmup 0 --cpu-baseline 0
[ -z "$SKIP" ] && step pmc_sq2 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 bench.py --config $CFG --reports $NP --steps 1 --warmup 0 --cpu-baseline 0
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --config $CFG --reports $NP --steps 1 --warmup 0 --cpu-baseline 0
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --config $CFG --reports $NP --steps 1 --warmup 0 --cpu-baseline 0
echo done >> "$OUT/steps.txt"
