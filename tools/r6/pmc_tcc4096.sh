#!/bin/bash
# round 6: L2 hit / miss counters of the B=4096 SAC step (one pass, kernel
# trace only) -> gpurun_out/r6/pmctcc
R=$PWD
O=$R/gpurun_out/r6/pmctcc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/tcc \
  -- python3 $R/bench.py --batch 4096 --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 > $O/tcc.log 2>&1
echo "pass tcc rc=$?"
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/ea \
  -- python3 $R/bench.py --batch 4096 --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 > $O/ea.log 2>&1
echo "pass ea rc=$?"
