# round 6 session 12: what the top tree levels of a sweep miss cost (kernel trace per knob)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06_v16; mkdir -p $OUT
K=build/libmastic_knobs.so
t() { local name=$1; shift; timeout -k 10 300 env "$@" rocprofv3 --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 tools/tiny_level_probe.py $K 12 380000 > $OUT/$name.log 2>&1; local rc=$?; tail -1 $OUT/$name.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc; return 0; }
t base X=1
t noproof MASTIC_DBG_SKIP=1
t nosponge MASTIC_DBG_SKIP=4
t nosplit MASTIC_SMALL_SPLIT=0
t noaes MASTIC_DBG_SKIP=2
echo done > $OUT/done.txt
