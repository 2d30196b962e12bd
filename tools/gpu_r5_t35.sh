#!/bin/bash
# round 5, final tree: policy-head column chunks at B=256 (OAC_HEAD_CC; the
# rule gives 4), interleaved
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2 3; do for cc in 0 2 8; do
  if [ $cc = 0 ]; then unset OAC_HEAD_CC; else export OAC_HEAD_CC=$cc; fi
  timeout -k 10 120 python tools/launch_times.py --batch 256 --rate-steps 1000 > gpurun_out/r5_t35_cc$cc.txt 2>&1; rc=$?; crash $rc
  echo "cc$cc | $(grep drop-in gpurun_out/r5_t35_cc$cc.txt | cut -c1-60) | $(grep -E 'launch +2 ' gpurun_out/r5_t35_cc$cc.txt | tr -s ' ')"
done; done
