set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v3; mkdir -p $OUT
timeout -k 5 60 python -u tools/comm_timeout_probe.py > $OUT/comm_probe.log 2>&1; rc=$?; grep -v "^\s*$" $OUT/comm_probe.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/timing_fix_ab.py > $OUT/timing_fix_ab.log 2>&1; rc=$?; cat $OUT/timing_fix_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_queued_calls.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/ptests.log 2>&1; rc=$?; tail -3 $OUT/ptests.log; exit $rc
