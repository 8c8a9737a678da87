set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_v23
timeout -k 10 300 python3 -m cProfile -s tottime bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_v23/c3sweep_cprofile.txt 2>&1
