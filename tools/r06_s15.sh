set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v15; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc; return 0; }
run bench_default 700 python3 -u bench.py
run c4 400 python3 -u bench.py --config c4 --cpu-baseline 0
run c5 400 python3 -u bench.py --config c5 --cpu-baseline 0
run c3sweep 400 python3 -u bench.py --config c3sweep --steps 1 --warmup 1 --cpu-baseline 0
echo done >> $OUT/steps.txt
