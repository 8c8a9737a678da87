# round 6 session 4: the driver's default bench, the wave-uniform-key AES microbenchmark,
# and the virtual-rank strong-scaling prediction of the north_star job on this library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v4; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -2 $OUT/$name.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc; return 0; }
AES_MB_TT_ONLY=1 run aes_mb 120 tools/aes_bs_mb
run bench_default 600 python3 -u bench.py
for k in 2 4 8; do run vr$k 300 python3 -u bench.py --config c2sweep --virtual-ranks $k --steps 1 --warmup 1 --cpu-baseline 0; done
echo done >> $OUT/steps.txt
