#!/bin/bash
# round 5, after the round-robin XCD mapping: its chunk size (2 / 4 / 8
# tiles), the backward tile config (OAC_BWDP_CFG 12 default / 10 / 9) and the
# split-K counts (OAC_SPLITS q1,q0,ph,p1,p0), interleaved on one box
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
L=$PWD/oac-explore_amd/oac_amd
run() {   # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 400 > gpurun_out/r5_t28_poac_$tag.txt 2>&1; rc=$?; crash $rc
  env "$@" timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 400 > gpurun_out/r5_t28_b4096_$tag.txt 2>&1; rc=$?; crash $rc
  echo "$tag | poac $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t28_poac_$tag.txt) | b4096 $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t28_b4096_$tag.txt)"
}
for r in 1 2; do
  run c2 OAC_LIB=$L/liboac_amd_c2.so
  run base OAC_LIB=$L/liboac_amd_base.so
  run c8 OAC_LIB=$L/liboac_amd_c8.so
  run bwd10 OAC_BWDP_CFG=10
  run bwd9 OAC_BWDP_CFG=9
  run sq0_16 OAC_SPLITS=0,16,0,0,0
  run sq0_8 OAC_SPLITS=0,8,0,0,0
  run sq1_8 OAC_SPLITS=8,0,0,0,0
  run sp_8 OAC_SPLITS=0,0,0,8,8
  run sp0_32 OAC_SPLITS=0,0,0,0,32
done
