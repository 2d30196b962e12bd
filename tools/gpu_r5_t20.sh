#!/bin/bash
# round 5: per-stage clocks of the large-batch forward (B=4096 Humanoid and
# configs[4]'s Ant dims) and backward kernels -- where a launch's time goes
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
O=gpurun_out/r5_t20_clocks.txt; : > $O
for tile in 128,64 128,128 64,64; do
  echo "== humanoid tile $tile" >> $O
  OAC_FWD2_TILE=$tile timeout -k 10 60 tools/micro/fwd_clock_micro 4096 376 17 256 >> $O 2>&1; rc=$?; crash $rc
  echo "== ant tile $tile" >> $O
  OAC_FWD2_TILE=$tile timeout -k 10 60 tools/micro/fwd_clock_micro 4096 111 8 256 >> $O 2>&1; rc=$?; crash $rc
done
echo "== bwd 10 (64x64)" >> $O
timeout -k 10 60 tools/micro/bwd_clock_micro 10 >> $O 2>&1; rc=$?; crash $rc
cat $O
