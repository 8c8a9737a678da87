#!/bin/bash
# Instruction-cache counters for the level kernels (one rocprofv3 pass).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${PROF_OUT:-gpurun_out/prof_icache}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_WAVE_CYCLES -d $OUT/ic -o run --output-format csv -- python3 bench.py --reports ${PMC_REPORTS:-4096} --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/ic.log 2>&1
echo "rc=$?" >> $OUT/ic.log
