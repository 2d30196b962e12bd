#!/bin/bash
mkdir -p gpurun_out
for v in "OAC_RG_PIPE=0" "OAC_RG_PIPE=1" "OAC_RG_PIPE=0" "OAC_RG_PIPE=1"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 10 --rate-steps 4000 > gpurun_out/lt256_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/lt256_$v.log | tail -13 | head -2
done
