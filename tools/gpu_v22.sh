set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_v22
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v22_gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v22_smoke.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/v22_c3sweep.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c1sweep > gpurun_out/v22_c1sweep.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/v22_c2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v22/c2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_v22/c2_stats.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v22/c3sweep -o run --output-format csv -- python3 bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_v22/c3sweep_stats.log 2>&1
