set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier_cache.py tests/test_gpu_sweep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/v13_fc_tests.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v13_gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3sweep --reports 16384 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/v13_c3sweep_16384.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c1sweep > gpurun_out/v13_c1sweep.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config c3sweep --reports 65536 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/v13_c3sweep_65536.log 2>&1
