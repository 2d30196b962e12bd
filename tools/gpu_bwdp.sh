#!/bin/bash
# LDS-DMA pipelined backward GEMM (gemm_bwdp.hip) against gemm_bwd.hip at the
# B=4096 SAC step's backward launches (tools/micro/bwd_micro); CLOCK=1: the
# clocked build (per-stage cycles of wave 0)
mkdir -p gpurun_out
BIN=tools/micro/bwd_micro
[ -n "$CLOCK" ] && BIN=tools/micro/bwd_clock_micro
for C in ${CFGS:-9 10 11}; do
  echo "== cfg $C"
  timeout -k 5 60 $BIN $C || exit $?
done 2>&1 | tee gpurun_out/bwdp.log
