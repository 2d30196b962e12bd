#!/bin/bash
# round 5: forward kernel with the masked stage as an instantiation of its own
# (k groups wholly outside the range skipped) -- clocks, parity, A/B
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
O=gpurun_out/r5_t24_clocks.txt; : > $O
for tile in 128,64 64,64; do
  echo "== humanoid tile $tile" >> $O
  OAC_FWD2_TILE=$tile timeout -k 10 60 tools/micro/fwd_clock_micro 4096 376 17 256 >> $O 2>&1; rc=$?; crash $rc
  echo "== ant tile $tile" >> $O
  OAC_FWD2_TILE=$tile timeout -k 10 60 tools/micro/fwd_clock_micro 4096 111 8 256 >> $O 2>&1; rc=$?; crash $rc
done
cat $O
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_particle.py tests/test_gpu_parity.py -x -q $T > gpurun_out/r5_t24_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t24_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5_t24_tests.log | head -20; exit $rc; }
PREV=$PWD/oac-explore_amd/oac_amd/liboac_amd_prev.so
for r in 1 2; do for v in prev cur; do
  if [ $v = prev ]; then export OAC_LIB=$PREV; else unset OAC_LIB; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > gpurun_out/r5_t24_poac_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v poac: $(grep drop-in gpurun_out/r5_t24_poac_$v.txt | cut -c1-60) | $(grep -E 'launch +[0135] ' gpurun_out/r5_t24_poac_$v.txt | tr -s ' ' | tr '\n' ' ')"
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t24_b4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t24_b4096_$v.txt | cut -c1-60) | $(grep -E 'launch +[013] ' gpurun_out/r5_t24_b4096_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
