#!/bin/bash
# round 5: why sac_humanoid_b4096's teacher step 2 fails with the chunked slab
# order (diag_teacher_flip), then the Adam-launch A/B against the previous build
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u tools/diag_teacher_flip.py sac_humanoid_b4096 > gpurun_out/r5_t18_diag.txt 2>&1; rc=$?; crash $rc
cat gpurun_out/r5_t18_diag.txt | tail -8
PREV=$PWD/oac-explore_amd/oac_amd/liboac_amd_prev.so
for r in 1 2; do for v in prev cur; do
  if [ $v = prev ]; then export OAC_LIB=$PREV; else unset OAC_LIB; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > gpurun_out/r5_t18_poac_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v poac: $(grep drop-in gpurun_out/r5_t18_poac_$v.txt | cut -c1-60) | $(grep 'adam' gpurun_out/r5_t18_poac_$v.txt | tr -s ' ' | tr '\n' ' ')"
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t18_b4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t18_b4096_$v.txt | cut -c1-60) | $(grep 'adam' gpurun_out/r5_t18_b4096_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
