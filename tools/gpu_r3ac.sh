#!/bin/bash
# backward tile A/B at B=4096 (SAC and configs[4]): 64x64 2-stage (default, cfg 12) against 128x64 / 64x128 on the 2-stage ring (cfg 13 / 14)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bwd_tiles.txt
for C in 12 13 14; do
  for P in "" "--poac"; do
    OAC_BWDP_CFG=$C timeout -k 10 120 python tools/launch_times.py --batch 4096 $P > gpurun_out/bt.txt 2>&1 || { cat gpurun_out/bt.txt; exit 1; }
    echo "OAC_BWDP_CFG=$C $P" >> gpurun_out/bwd_tiles.txt
    grep -v amdgpu.ids gpurun_out/bt.txt >> gpurun_out/bwd_tiles.txt
  done
done
grep "OAC_BWDP\|drop-in" gpurun_out/bwd_tiles.txt
