#!/bin/bash
# A/B timing: GPU tests with the default build, then the C2 bench for the
# default build, each build/lib*.so variant (bench.py --lib) and each
# "NAME=ENV=VALUE" entry of $AB_ENVS.
set -o pipefail
if [ -z "$AB_NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
fi
for R in ${AB_REPORTS:-8192 4096}; do
  timeout -k 10 200 python bench.py --reports $R --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/ab_default_$R.json || exit $?
  for f in build/lib*.so; do
    [ -e "$f" ] || continue
    v=$(basename $f .so)
    timeout -k 10 200 python bench.py --lib $PWD/$f --reports $R --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/ab_${v}_$R.json || exit $?
  done
  for e in $AB_ENVS; do
    name=${e%%=*}; kv=${e#*=}
    env "$kv" timeout -k 10 200 python bench.py --reports $R --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/ab_${name}_$R.json || exit $?
  done
done
