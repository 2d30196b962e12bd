#!/bin/bash
# round 5: the targets kernel's last-layer dW on 16-column groups (256 blocks
# at B=4096 instead of 128) -- parity, then A/B against the build before
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_parity.py tests/test_gpu_dp.py -x -q $T > gpurun_out/r5_t36_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t36_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5_t36_tests.log | head -20; exit $rc; }
L=$PWD/oac-explore_amd/oac_amd
for r in 1 2 3; do for v in base cur; do
  if [ $v = cur ]; then unset OAC_LIB; else export OAC_LIB=$L/liboac_amd_$v.so; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t36_b4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t36_b4096_$v.txt | cut -c1-60) | $(grep -E 'launch +4 ' gpurun_out/r5_t36_b4096_$v.txt | tr -s ' ')"
done; done
