set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_v25
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v25/c3sweep131k -o run --output-format csv -- python3 bench.py --config c3sweep --reports 131072 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_v25/stats.log 2>&1
