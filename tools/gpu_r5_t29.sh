#!/bin/bash
# round 5: B=4096 SAC split-K counts of the critic layer-0 dW (q0) and the
# policy layer-0 dW (p0) after the round-robin XCD mapping (OAC_SPLITS)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 400 > gpurun_out/r5_t29_b4096_$tag.txt 2>&1; rc=$?; crash $rc
  echo "$tag | b4096 $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t29_b4096_$tag.txt) | $(grep -E 'launch +(6|7|11) ' gpurun_out/r5_t29_b4096_$tag.txt | tr -s ' ' | tr '\n' ' ')"
}
for r in 1 2; do
  run base OAC_X=0
  run q0_4 OAC_SPLITS=0,4,0,0,0
  run q0_6 OAC_SPLITS=0,6,0,0,0
  run q0_8 OAC_SPLITS=0,8,0,0,0
  run q0_10 OAC_SPLITS=0,10,0,0,0
  run p0_8 OAC_SPLITS=0,0,0,0,8
  run p0_12 OAC_SPLITS=0,0,0,0,12
  run q0_8p0_12 OAC_SPLITS=0,8,0,0,12
done
