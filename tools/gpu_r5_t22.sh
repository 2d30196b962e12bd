#!/bin/bash
# round 5: LDS ring depth of the 128x64 forward tile (NB = 2: 48 KB, three
# workgroups per CU; 3: 72 KB, two) by launch size -- stage clocks, then the step
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
O=gpurun_out/r5_t22_clocks.txt; : > $O
for nb in 2 3; do
  echo "== humanoid 128,64 NB=$nb" >> $O
  OAC_FWD2_NB=$nb OAC_FWD2_TILE=128,64 timeout -k 10 60 tools/micro/fwd_clock_micro 4096 376 17 256 >> $O 2>&1; rc=$?; crash $rc
  echo "== ant 128,64 NB=$nb" >> $O
  OAC_FWD2_NB=$nb OAC_FWD2_TILE=128,64 timeout -k 10 60 tools/micro/fwd_clock_micro 4096 111 8 256 >> $O 2>&1; rc=$?; crash $rc
done
cat $O
for r in 1 2; do for nb in 0 3; do
  if [ $nb = 0 ]; then unset OAC_FWD2_NB; else export OAC_FWD2_NB=$nb; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > gpurun_out/r5_t22_poac_$nb.txt 2>&1; rc=$?; crash $rc
  echo "nb$nb poac: $(grep drop-in gpurun_out/r5_t22_poac_$nb.txt | cut -c1-60) | $(grep -E 'launch +[013589] ' gpurun_out/r5_t22_poac_$nb.txt | tr -s ' ' | tr '\n' ' ')"
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t22_b4096_$nb.txt 2>&1; rc=$?; crash $rc
  echo "nb$nb b4096: $(grep drop-in gpurun_out/r5_t22_b4096_$nb.txt | cut -c1-60) | $(grep -E 'launch +[013] ' gpurun_out/r5_t22_b4096_$nb.txt | tr -s ' ' | tr '\n' ' ')"
done; done
