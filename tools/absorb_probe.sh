#!/bin/bash
# Absorb-kernel probe: serialized C2 bench at 8192 reports with plane-row pad 0 and 64,
# plus one PMC pass each (cache hit/miss, fetch) over a 1-step run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/absorb_probe
mkdir -p $OUT
for P in 0 64; do
  AMD_SERIALIZE_KERNEL=3 MASTIC_STRIDE_PAD=$P timeout -k 10 300 python bench.py --reports 8192 --steps 1 --warmup 1 --cpu-baseline 0 > $OUT/ser_pad$P.json || exit $?
done
for P in 0 64; do
  MASTIC_STRIDE_PAD=$P timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $OUT/pmc_pad$P -o run --output-format csv -- python3 bench.py --reports 8192 --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_pad$P.log 2>&1 || exit $?
done
