set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_v8; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0 > $O/c3sweep_fused.log 2>&1 || exit 1
MASTIC_FUSE_PROOFS=0 timeout -k 10 300 python3 bench.py --config c3sweep --steps 1 --warmup 0 --cpu-baseline 0 > $O/c3sweep_nofuse.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --config c2sweep --steps 1 --warmup 0 --cpu-baseline 0 > $O/c2sweep.log 2>&1 || exit 1
echo done
