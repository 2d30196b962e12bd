#!/bin/bash
# round 5: split-K counts against the Adam launches' slab reads -- configs[4]
# (P-OAC K=10, Ant dims, B=4096) and the B=4096 SAC step, OAC_SPLITS="q1,q0,ph,p1,p0"
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
out=gpurun_out/r5_t10_splits.txt; : > $out
for S in "0,0,0,0,0" "0,16,0,0,0" "0,8,0,0,0" "0,0,0,0,16" "0,0,0,0,8" "0,0,16,0,0" "0,0,8,0,0" "8,0,0,8,0" "0,16,16,0,16" "0,0,0,0,0"; do
  echo "== poac OAC_SPLITS=$S" >> $out
  OAC_SPLITS=$S timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 --steps 10 --rate-steps 1000 > gpurun_out/r5_t10_tmp.txt 2>&1; rc=$?; crash $rc
  grep -v amdgpu.ids gpurun_out/r5_t10_tmp.txt >> $out; echo "poac $S: $(grep drop-in gpurun_out/r5_t10_tmp.txt)"
done
for S in "0,0,0,0,0" "0,0,0,0,8" "0,0,0,8,8" "0,8,0,0,0"; do
  echo "== sac OAC_SPLITS=$S" >> $out
  OAC_SPLITS=$S timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 1000 > gpurun_out/r5_t10_tmp.txt 2>&1; rc=$?; crash $rc
  grep -v amdgpu.ids gpurun_out/r5_t10_tmp.txt >> $out; echo "sac $S: $(grep drop-in gpurun_out/r5_t10_tmp.txt)"
done
