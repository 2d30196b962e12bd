#!/bin/bash
# forward ring depth for 128x64 tiles: OAC_FWD2_NB=3 vs default 2 (per-launch)
mkdir -p gpurun_out
for v in "OAC_FWD2_NB=0" "OAC_FWD2_NB=3"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ltnb_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/ltnb_$v.log | tail -16 | sed -n '1p;3,4p;6p'
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ltnbp_$v.log 2>&1 || exit $?
  grep -v "^launch" gpurun_out/ltnbp_$v.log | tail -19 | sed -n '1p;3,4p;6p;11,12p'
done
