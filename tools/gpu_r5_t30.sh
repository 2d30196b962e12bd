#!/bin/bash
# round 5: power-of-two split-K counts for the pipelined backward dW (B=4096
# SAC critic layer 0: 13 -> 8) -- parity, then A/B against the build before
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_particle.py tests/test_gpu_parity.py tests/test_gpu_altkernels.py tests/test_gpu_dp.py -x -q $T > gpurun_out/r5_t30_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t30_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5_t30_tests.log | head -20; exit $rc; }
L=$PWD/oac-explore_amd/oac_amd
for r in 1 2; do for v in base cur; do
  if [ $v = cur ]; then unset OAC_LIB; else export OAC_LIB=$L/liboac_amd_$v.so; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t30_b4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t30_b4096_$v.txt | cut -c1-60)"
done; done
# forward tile per launch after the round-robin XCD mapping: every forward
# launch forced to 128x64 / 64x64 (OAC_FWD2_TILE) against the rule's choice
for t in rule 128,64 64,64; do
  if [ $t = rule ]; then unset OAC_FWD2_TILE; else export OAC_FWD2_TILE=$t; fi
  n=${t/,/x}
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 400 > gpurun_out/r5_t30_tile_poac_$n.txt 2>&1; rc=$?; crash $rc
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 400 > gpurun_out/r5_t30_tile_b4096_$n.txt 2>&1; rc=$?; crash $rc
done
unset OAC_FWD2_TILE
for n in rule 128x64 64x64; do echo "== $n"; paste gpurun_out/r5_t30_tile_b4096_$n.txt gpurun_out/r5_t30_tile_poac_$n.txt | grep -E "drop-in|gemm" | tr -s ' ' | cut -c1-100; done
