# ad-hoc GPU session (edited per experiment; see tools/gpu_session.sh for the standard steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_v10; mkdir -p $O
run() { local n=$1; shift; echo "[$(date +%T)] $n" >> $O/steps.txt; timeout -k 10 600 "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?" >> $O/steps.txt; tail -5 $O/$n.log; exit 1; }; }
run c2sweep_nofuse env MASTIC_FUSE_PROOFS=0 python3 bench.py --config c2sweep --steps 1 --warmup 0 --cpu-baseline 0
run c3sweep_131072 python3 bench.py --config c3sweep --reports 131072 --steps 1 --warmup 0 --cpu-baseline 0
run stats_c3sweep_131072 rocprofv3 --kernel-trace --stats -d $O/stats_c3sweep_131072 -o run --output-format csv -- python3 bench.py --config c3sweep --reports 131072 --steps 1 --warmup 0 --cpu-baseline 0
rm -f $O/stats_c3sweep_131072/run_kernel_trace.csv.gz
echo done >> $O/steps.txt
