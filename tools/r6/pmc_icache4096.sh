#!/bin/bash
# round 6: instruction-cache counters of the B=4096 SAC step (one pass,
# kernel trace only) -> gpurun_out/r6/pmcic
R=$PWD
O=$R/gpurun_out/r6/pmcic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/ic \
  -- python3 $R/bench.py --batch 4096 --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 > $O/ic.log 2>&1
echo "pass ic rc=$?"
