#!/bin/bash
# policy-head workgroups per row block at B=256 (OAC_HEAD_CC)
mkdir -p gpurun_out
for v in 4 2 8 4; do
  OAC_HEAD_CC=$v timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 10 --rate-steps 4000 > gpurun_out/lthc_$v.log 2>&1 || exit $?
  echo "cc=$v: $(grep drop-in gpurun_out/lthc_$v.log) $(grep 'launch  2' gpurun_out/lthc_$v.log)"
done
