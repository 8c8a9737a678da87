# round 6 session 10: occupancy of the one-lane binder sponges beside the level kernel on the north_star
# sweep (knob build): LDS reserved per sponge workgroup (MASTIC_ABSORB_LDS_KB, caps sponge workgroups per
# CU; 10 KB leaves one beside a 150 KB level-kernel workgroup) and smaller sponge workgroups
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v10; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -1 $OUT/$name.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc; return 0; }
SW="--config c2sweep --steps 1 --warmup 1 --cpu-baseline 0 --standalone 0 --lib build/libmastic_knobs.so"
for rep in 1 2; do
  run base_$rep 300 python3 -u bench.py $SW
  MASTIC_ABSORB_LDS_KB=10 run lds10_$rep 300 python3 -u bench.py $SW
  MASTIC_ABSORB_LDS_KB=40 run lds40_$rep 300 python3 -u bench.py $SW
  MASTIC_ABSORB_THREADS=64 run thr64_$rep 300 python3 -u bench.py $SW
done
echo done >> $OUT/steps.txt
