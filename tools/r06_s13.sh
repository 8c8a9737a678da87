# round 6 session 13: the level kernel's prologue (table fill from a compile-time T0 table by
# wave-uniform scalar loads, key-schedule loads issued together): parity, then same-box A/B vs
# the library before it (build/libmastic_prefill.so), then the tiny-level trace again
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v13; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc; return 0; }
run parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rejection.py tests/test_gpu_frontier_cache.py tests/test_gpu_fill_offsets.py -m gpu -x -q --timeout 120 --timeout-method thread
SW="--config c2sweep --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0"
C2="--config c2 --steps 3 --warmup 1 --north-star 0 --full-job 0 --cpu-baseline 0 --standalone 0"
for rep in 1 2; do
  run sw_new_$rep 300 python3 -u bench.py $SW
  run sw_old_$rep 300 python3 -u bench.py $SW --lib build/libmastic_prefill.so
  run c2_new_$rep 300 python3 -u bench.py $C2
  run c2_old_$rep 300 python3 -u bench.py $C2 --lib build/libmastic_prefill.so
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/probe -o run --output-format csv -- python3 tools/tiny_level_probe.py '' 12 380000 > $OUT/probe.log 2>&1
echo done >> $OUT/steps.txt
