# round 6 session 9: C5 at its per-GPU job size (8M reports = 64M / 8 GPUs, cycled pool of 2^16) on the
# final round-6 library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v22; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc; return 0; }
run c5_8M 1000 python3 -u bench.py --config c5 --total-reports 8000000 --pool-reports 65536 --full-job 1 --cpu-baseline 0 --standalone 0
echo done >> $OUT/steps.txt
