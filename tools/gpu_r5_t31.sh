#!/bin/bash
# round 5, on the final tree: the remaining plan switches re-swept after the
# XCD mapping and split changes -- policy-head column chunks (OAC_HEAD_CC),
# the particle critic's dh2 in the targets kernel (OAC_DH2_TARGETS), the split
# Adam schedule at B=4096 (OAC_SPLIT_ADAM)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 400 > gpurun_out/r5_t31_poac_$tag.txt 2>&1; rc=$?; crash $rc
  env "$@" timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 400 > gpurun_out/r5_t31_b4096_$tag.txt 2>&1; rc=$?; crash $rc
  echo "$tag | poac $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t31_poac_$tag.txt) | b4096 $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t31_b4096_$tag.txt) | b4096 head $(grep -E 'launch +2 ' gpurun_out/r5_t31_b4096_$tag.txt | tr -s ' ')"
}
for r in 1 2; do
  run base OAC_X=0
  run cc2 OAC_HEAD_CC=2
  run cc4 OAC_HEAD_CC=4
  run nodh2 OAC_DH2_TARGETS=0
  run nosplitadam OAC_SPLIT_ADAM=0
done
