#!/bin/bash
# A/B timing: GPU tests with the default build, then the C2 bench for the
# default build and for each build/lib*.so variant (MASTIC_LIB override).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for R in ${AB_REPORTS:-8192 4096}; do
  timeout -k 10 200 python bench.py --reports $R --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/ab_default_$R.json || exit $?
  for f in build/lib*.so; do
    [ -e "$f" ] || continue
    v=$(basename $f .so)
    MASTIC_LIB=$PWD/$f timeout -k 10 200 python bench.py --reports $R --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/ab_${v}_$R.json || exit $?
  done
done
