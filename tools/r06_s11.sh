# round 6 session 11: kernel trace of one north_star sweep (per-launch durations by tree level)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v11; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --config c2sweep --steps 1 --warmup 0 --cpu-baseline 0 --standalone 0 > $OUT/bench.log 2>&1; rc=$?
tail -1 $OUT/bench.log | cut -c1-200
ls -la $OUT/trace
exit $rc
