# ad-hoc GPU session (edited per experiment; see tools/gpu_session.sh for the standard steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_v14; mkdir -p $O
run() { local n=$1; shift; echo "[$(date +%T)] $n" >> $O/steps.txt; timeout -k 10 900 "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?" >> $O/steps.txt; tail -15 $O/$n.log; exit 1; }; }
B="python3 bench.py --config c2 --steps 4 --warmup 1 --cpu-baseline 0 --full-job 0 --total-reports 12288"
NT=$PWD/draft-mouris-cfrg-mastic_amd/mastic_amd/libmastic_hip_nt.so
for i in 1 2; do
run base_$i $B
run nt_$i $B --lib $NT
done
run c5_nt python3 bench.py --config c5 --steps 3 --warmup 1 --cpu-baseline 0 --lib $NT
run c5_base python3 bench.py --config c5 --steps 3 --warmup 1 --cpu-baseline 0
echo done >> $O/steps.txt
