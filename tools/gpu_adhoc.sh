# ad-hoc GPU session (edited per experiment; see tools/gpu_session.sh for the standard steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_v12; mkdir -p $O
run() { local n=$1; shift; echo "[$(date +%T)] $n" >> $O/steps.txt; timeout -k 10 900 "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?" >> $O/steps.txt; tail -15 $O/$n.log; exit 1; }; }
run tests python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15
run c2sweep python3 bench.py --config c2sweep --steps 1 --warmup 0 --cpu-baseline 0
run c3sweep python3 bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0
for c in c5 c4; do
run ${c}_pw16 python3 bench.py --config $c --steps 3 --warmup 1 --cpu-baseline 0
run ${c}_pw8 env MASTIC_PAR_WAVES=8 MASTIC_SPLIT_ELEMS=0 python3 bench.py --config $c --steps 3 --warmup 1 --cpu-baseline 0
done
run c5_nosplit env MASTIC_SPLIT_ELEMS=0 python3 bench.py --config c5 --steps 3 --warmup 1 --cpu-baseline 0
B="python3 bench.py --config c2 --steps 4 --warmup 1 --cpu-baseline 0 --full-job 0 --total-reports 24576"
run c2_pw8 $B
run c2_pw16 env MASTIC_PAR_WAVES=16 $B
run c2_24576 python3 bench.py --config c2 --reports 24576 --steps 2 --warmup 1 --cpu-baseline 0 --full-job 0 --total-reports 49152
echo done >> $O/steps.txt
