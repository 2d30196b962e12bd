#!/bin/bash
# B=4096 SAC drop-in step rate by forced split-K counts (OAC_SPLITS="q1,q0,ph,p1,p0")
mkdir -p gpurun_out
for S in ${SPLITS:-"16,13,0,16,16" "16,10,0,16,16" "16,13,0,12,12" "16,13,0,20,20" "12,13,0,16,16" "20,13,0,16,16" "16,13,16,16,16" "16,16,0,16,16"}; do
  echo "== OAC_SPLITS=$S"
  OAC_SPLITS=$S timeout -k 5 100 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 300 2>&1 | grep -v amdgpu.ids | head -1 || exit $?
done 2>&1 | tee gpurun_out/split_bwdp.log
