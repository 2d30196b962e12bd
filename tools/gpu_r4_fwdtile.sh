#!/bin/bash
# per-launch forward tile A/B at configs[4] and B=4096 SAC (OAC_FWD2_TILE forces one tile shape)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for t in "" "64,64" "128,64"; do
  for w in "--batch 4096 --poac" "--batch 4096"; do
    OAC_FWD2_TILE=$t timeout -k 10 200 python tools/launch_times.py $w > gpurun_out/r4_ft.log 2>&1; crash $?
    echo "tile=[$t] $w"; grep -v amdgpu gpurun_out/r4_ft.log | head -6
  done
done
