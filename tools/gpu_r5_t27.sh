#!/bin/bash
# round 5: the critic layer 0's rank continuation staged by the main pipe (its
# loads under the last stage and the first epilogue) -- clocks, parity, A/B
# against the build before it (liboac_amd_base.so)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
O=gpurun_out/r5_t27_clocks.txt; : > $O
echo "== humanoid 128,64" >> $O
OAC_FWD2_TILE=128,64 timeout -k 10 60 tools/micro/fwd_clock_micro 4096 376 17 256 >> $O 2>&1; rc=$?; crash $rc
echo "== ant 128,64" >> $O
OAC_FWD2_TILE=128,64 timeout -k 10 60 tools/micro/fwd_clock_micro 4096 111 8 256 >> $O 2>&1; rc=$?; crash $rc
grep -A1 "layer0" $O | cut -c1-240
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_particle.py tests/test_gpu_parity.py tests/test_gpu_altkernels.py -x -q $T > gpurun_out/r5_t27_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t27_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5_t27_tests.log | head -20; exit $rc; }
L=$PWD/oac-explore_amd/oac_amd
for r in 1 2; do for v in base cur; do
  if [ $v = cur ]; then unset OAC_LIB; else export OAC_LIB=$L/liboac_amd_$v.so; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > gpurun_out/r5_t27_poac_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v poac: $(grep drop-in gpurun_out/r5_t27_poac_$v.txt | cut -c1-60) | $(grep -E 'launch +0 ' gpurun_out/r5_t27_poac_$v.txt | tr -s ' ')"
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t27_b4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t27_b4096_$v.txt | cut -c1-60) | $(grep -E 'launch +[013] ' gpurun_out/r5_t27_b4096_$v.txt | tr -s ' ' | tr '\n' ' ')"
done; done
