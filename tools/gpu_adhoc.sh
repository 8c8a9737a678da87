# ad-hoc GPU session (edited per experiment; see tools/gpu_session.sh for the standard steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_v11; mkdir -p $O
run() { local n=$1; shift; echo "[$(date +%T)] $n" >> $O/steps.txt; timeout -k 10 600 "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?" >> $O/steps.txt; tail -5 $O/$n.log; exit 1; }; }
B="python3 bench.py --config c2 --steps 5 --warmup 1 --cpu-baseline 0 --full-job 0 --total-reports 12288"
for i in 1 2; do
run base_$i $B
run single_$i env MASTIC_ABSORB_SINGLE=1 $B
run prio0_$i env MASTIC_ABSORB_PRIO=0 $B
run single_prio0_$i env MASTIC_ABSORB_SINGLE=1 MASTIC_ABSORB_PRIO=0 $B
done
echo done >> $O/steps.txt
