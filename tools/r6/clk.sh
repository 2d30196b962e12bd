#!/bin/bash
# stage clocks of the backward kernel (tools/micro/bwd_clock_micro, built from
# the current gemm_bwdp.hip) for cfg $CFG
O=$PWD/gpurun_out/r6/${TAG:-clk}
mkdir -p $O
timeout -k 5 60 tools/micro/bwd_clock_micro ${CFG:-12} 1 > $O/clock_${CFG:-12}.txt 2>&1 || exit $?
paste -d' ' <(grep -v clocks $O/clock_${CFG:-12}.txt | cut -c1-34) <(grep clocks $O/clock_${CFG:-12}.txt | cut -c1-220)
