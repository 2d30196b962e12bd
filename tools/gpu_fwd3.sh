#!/bin/bash
# LDS-pipelined forward GEMM (gemm_fwd.hip) against the register-direct kernel:
# bitwise comparison + per-launch time by tile (tools/micro/fwd_micro);
# FWD_CLOCK=1: the clocked build (per-stage cycles of wave 0)
mkdir -p gpurun_out
BIN=tools/micro/fwd_micro
[ -n "$FWD_CLOCK" ] && BIN=tools/micro/fwd_clock_micro
for T in ${TILES:-128,128 128,64 64,128 64,64}; do
  echo "== OAC_FWD2_TILE=$T"
  OAC_FWD2_TILE=$T timeout -k 5 60 $BIN ${1:-4096} || exit $?
done 2>&1 | tee gpurun_out/fwd3.log
