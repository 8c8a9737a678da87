#!/bin/bash
# kernel traces of the C2 bench at 8192 reports, plane pad 0 vs 64
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for P in 0 64; do
  MASTIC_STRIDE_PAD=$P timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/atrace_pad$P -o run --output-format csv -- python3 bench.py --reports 8192 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/atrace_pad$P.log 2>&1 || exit $?
done
