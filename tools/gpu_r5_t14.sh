#!/bin/bash
# round 5: GemmBatch records in device memory (BatchCache) against the
# by-value kernel arguments -- B=256 parity subset, then interleaved A/B of
# the steady rate, the per-launch durations and the driver's window
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ring.py tests/test_gpu_particle.py -x -q $T > gpurun_out/r5_t14_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t14_tests.log; [ $rc -eq 0 ] || exit $rc
PREV=$PWD/oac-explore_amd/oac_amd/liboac_amd_prev.so
for r in 1 2; do for v in prev cur; do
  if [ $v = prev ]; then export OAC_LIB=$PREV; else unset OAC_LIB; fi
  timeout -k 10 120 python tools/launch_times.py > gpurun_out/r5_t14_lt_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v: $(grep drop-in gpurun_out/r5_t14_lt_$v.txt | cut -c1-90)"
  grep launch gpurun_out/r5_t14_lt_$v.txt | grep -v drop | awk '{printf "%s ", $4}'; echo
  for i in 1 2; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r5_t14_drv.json 2>/dev/null; rc=$?; crash $rc
    python -c "import json; d=json.loads(open('gpurun_out/r5_t14_drv.json').read().strip().splitlines()[-1]); print('  driver shape', d['value'])"
  done
done; done
for v in prev cur; do
  if [ $v = prev ]; then export OAC_LIB=$PREV; else unset OAC_LIB; fi
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --rate-steps 600 > gpurun_out/r5_t14_lt4096_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v b4096: $(grep drop-in gpurun_out/r5_t14_lt4096_$v.txt | cut -c1-90)"
  timeout -k 10 120 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > gpurun_out/r5_t14_ltpoac_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v poac: $(grep drop-in gpurun_out/r5_t14_ltpoac_$v.txt | cut -c1-90)"
done
