set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v12_gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v12_smoke.txt 2>&1 && \
PROF_OUT=gpurun_out/prof_v12 bash tools/profile_r01.sh
