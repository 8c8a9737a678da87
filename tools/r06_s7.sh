# round 6 session 7: binder-sponge wave priority on the north_star sweep (knob build, interleaved),
# then the other BASELINE configs' bench lines on the round-6 library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v7; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc; return 0; }
SW="--config c2sweep --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0 --lib build/libmastic_knobs.so"
for rep in 1 2; do
  for prio in 3 1 0; do MASTIC_ABSORB_PRIO=$prio run prio${prio}_$rep 300 python3 -u bench.py $SW; done
done
run c3sweep 400 python3 -u bench.py --config c3sweep --steps 1 --warmup 1 --cpu-baseline 0
run c4 400 python3 -u bench.py --config c4 --cpu-baseline 0
run c5 400 python3 -u bench.py --config c5 --cpu-baseline 0
run c1sweep 300 python3 -u bench.py --config c1sweep --cpu-baseline 0
echo done >> $OUT/steps.txt
