#!/bin/bash
# Kernel traces of one C2 / C4 step with the binder sponges' message loads on
# and off (MASTIC_ABSORB_DBG=1: permutations only, results wrong) through the
# experiment-knob build: how much of the lone last-level sponge chain after
# the last level kernel is load latency.  Output: gpurun_out/<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for cfg in c2 c4; do
for dbg in 0 1; do
  MASTIC_ABSORB_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/${cfg}_dbg$dbg" -o run --output-format csv -- \
    python3 bench.py --config $cfg --lib "$PWD/build/lib_knobs.so" --steps 1 --warmup 1 --north-star 0 --cpu-baseline 0 --full-job 0 \
    > "$OUT/${cfg}_dbg$dbg.log" 2>&1 || exit $?
done
done
echo done
