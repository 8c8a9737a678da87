set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 -k "not without_peers" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/timing_fix_ab.py > $OUT/timing_fix_ab.log 2>&1; rc=$?; cat $OUT/timing_fix_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 5 90 python -u tools/comm_timeout_probe.py > $OUT/comm_probe.log 2>&1; rc=$?; cat $OUT/comm_probe.log | tail -20; exit $rc
