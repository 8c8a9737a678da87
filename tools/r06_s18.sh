# round 6 session 18: strong-scaling prediction on the final kernel (same box, one session)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v18; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc; return 0; }
run vr1 300 python3 -u bench.py --config c2sweep --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0
for k in 2 4 8; do run vr$k 300 python3 -u bench.py --config c2sweep --virtual-ranks $k --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0; done
echo done >> $OUT/steps.txt
