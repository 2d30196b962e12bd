#!/bin/bash
# round 5: which change slowed particle_min_kernel (r04 = base; A = r04 + the
# NaN-safe argmin; B = current (W_last rows staged through LDS))
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2; do for v in base A B; do
  L=$PWD/oac-explore_amd/oac_amd/liboac_amd_$v.so; [ $v = cur ] && L=$PWD/oac-explore_amd/oac_amd/liboac_amd.so
  OAC_LIB=$L timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 300 --poac > gpurun_out/r5_t7_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v: $(head -1 gpurun_out/r5_t7_$v.txt | cut -c1-60) | $(grep 'launch  4 \|launch 10 ' gpurun_out/r5_t7_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
