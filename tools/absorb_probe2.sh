#!/bin/bash
# serialized C2 bench (absorb time alone) for several reports:pad:absorb_lds_kb points
OUT=gpurun_out/absorb_probe2
mkdir -p $OUT
for spec in $SWEEP; do
  IFS=: read R P L <<< "$spec"
  AMD_SERIALIZE_KERNEL=3 MASTIC_STRIDE_PAD=$P MASTIC_ABSORB_LDS_KB=$L timeout -k 10 300 python bench.py --reports $R --steps 1 --warmup 1 --cpu-baseline 0 > $OUT/r${R}_pad${P}_lds$L.json || exit $?
done
