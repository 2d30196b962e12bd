#!/bin/bash
# round 5, final tree: the forward launches forced to 64x128 / 128x128 tiles
# against the per-launch rule (per-launch breakdowns)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2; do for t in rule 64,128 128,128; do
  if [ $t = rule ]; then unset OAC_FWD2_TILE; else export OAC_FWD2_TILE=$t; fi
  n=${t/,/x}
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 400 > gpurun_out/r5_t32_poac_$n.txt 2>&1; rc=$?; crash $rc
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 400 > gpurun_out/r5_t32_b4096_$n.txt 2>&1; rc=$?; crash $rc
  echo "$n | poac $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t32_poac_$n.txt) $(grep -E 'launch +(0|1|3|8|9) ' gpurun_out/r5_t32_poac_$n.txt | tr -s ' ' | cut -d' ' -f3,5 | tr '\n' ' ') | b4096 $(grep -o '[0-9.]* steps/s' gpurun_out/r5_t32_b4096_$n.txt) $(grep -E 'launch +(0|1|3) ' gpurun_out/r5_t32_b4096_$n.txt | tr -s ' ' | cut -d' ' -f3,5 | tr '\n' ' ')"
done; done
