#!/bin/bash
# round 5: configs[4] critic layer-0 dW launch 9.8 -> 13.0 us -- the earlier
# round-5 build against the current one on one box, and each one's launch shapes
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2; do for v in base cur; do
  L=$PWD/oac-explore_amd/oac_amd/liboac_amd_$v.so; [ $v = cur ] && L=$PWD/oac-explore_amd/oac_amd/liboac_amd.so
  OAC_LIB=$L timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 1000 --poac > gpurun_out/r5_t11_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v: $(grep drop-in gpurun_out/r5_t11_$v.txt | cut -c1-60) | $(grep 'launch  6 \|launch  5 ' gpurun_out/r5_t11_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
for v in base cur; do
  L=$PWD/oac-explore_amd/oac_amd/liboac_amd_$v.so; [ $v = cur ] && L=$PWD/oac-explore_amd/oac_amd/liboac_amd.so
  OAC_DEBUG_CFG=1 OAC_LIB=$L timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 2 --rate-steps 2 --poac > gpurun_out/r5_t11_cfg_$v.txt 2>&1; rc=$?; crash $rc
  grep "^launch" gpurun_out/r5_t11_cfg_$v.txt | head -40 | sort | uniq | head -20 | cut -c1-200
done
