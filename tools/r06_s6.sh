set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v6; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name" >> $OUT/steps.txt
        timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc" >> $OUT/steps.txt
        tail -2 $OUT/$name.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc; return 0; }
run ptests 400 python -u -m pytest tests/test_gpu_serial_sponges.py tests/test_gpu_comm.py -m gpu -x -v --timeout 120 --timeout-method thread
run bench_default 700 python3 -u bench.py
echo done >> $OUT/steps.txt
