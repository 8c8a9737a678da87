# round 6 session 17: key-schedule loads issued before the table fill (A/B vs build/libmastic_prekey.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v17; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc; return 0; }
run parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frontier_cache.py -m gpu -x -q --timeout 120 --timeout-method thread
SW="--config c2sweep --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0"
for rep in 1 2 3; do
  run sw_new_$rep 300 python3 -u bench.py $SW
  run sw_old_$rep 300 python3 -u bench.py $SW --lib build/libmastic_prekey.so
done
echo done >> $OUT/steps.txt
