#!/bin/bash
# round 5: per-stage clocks of the large-batch backward kernel (64x64 and 128x64)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
O=gpurun_out/r5_t26_bwd_clocks.txt; : > $O
for c in 10 9; do
  echo "== bwdp cfg $c" >> $O
  timeout -k 10 90 tools/micro/bwd_clock_micro $c 1 >> $O 2>&1; rc=$?; crash $rc
done
cat $O
