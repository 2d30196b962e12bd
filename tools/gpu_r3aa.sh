#!/bin/bash
# split-count sweep of the B=4096 SAC dW launches after the last-layer move (OAC_SPLITS="q1,q0,ph,p1,p0")
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/split_sweep.txt
for S in "0,0,0,0,0" "0,14,0,0,0" "0,15,0,0,0" "0,12,0,0,0" "0,0,0,0,20" "0,0,0,0,24" "0,0,0,20,0"; do
  OAC_SPLITS=$S timeout -k 10 120 python tools/launch_times.py --batch 4096 > gpurun_out/ss.txt 2>&1 || { cat gpurun_out/ss.txt; exit 1; }
  echo "OAC_SPLITS=$S" >> gpurun_out/split_sweep.txt
  grep -v amdgpu.ids gpurun_out/ss.txt >> gpurun_out/split_sweep.txt
done
grep -A0 "OAC_SPLITS\|drop-in" gpurun_out/split_sweep.txt
