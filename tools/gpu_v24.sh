set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c3sweep --reports 131072 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/v24_c3sweep_131072.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config c3sweep --reports 262144 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/v24_c3sweep_262144.log 2>&1
