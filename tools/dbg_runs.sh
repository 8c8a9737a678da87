set -e
for v in 0 1 3 4; do
  MASTIC_EVAL_DBG=$v timeout -k 10 120 python bench.py --reports 4096 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/dbg_$v.json
done
MASTIC_EVAL_QUAD=1 timeout -k 10 120 python bench.py --reports 4096 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/dbg_quad.json
for v in 0 4; do
  AMD_SERIALIZE_KERNEL=3 MASTIC_EVAL_DBG=$v timeout -k 10 120 python bench.py --reports 4096 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/dbg_ser_$v.json
done
