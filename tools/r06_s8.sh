# round 6 session 8: BASELINE configs at their per-GPU job sizes on the final round-6 library
# (C3: 2M reports = 16M / 8 GPUs, full pruned sweep; C4: 4M-report job over a cycled pool of 262,144)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v21; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc; return 0; }
run c3sweep_2M 400 python3 -u bench.py --config c3sweep --reports 2000000 --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0
run c4_4M 700 python3 -u bench.py --config c4 --total-reports 4000000 --pool-reports 262144 --full-job 1 --cpu-baseline 0 --standalone 0
echo done >> $OUT/steps.txt
