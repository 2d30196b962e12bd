#!/bin/bash
# round 5: A/B of the current tree against the previous build (liboac_amd_prev.so):
# parity first,
# then interleaved A/B against the previous build
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ring.py tests/test_gpu_dp.py -x -q $T > gpurun_out/r5_t16_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t16_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r5_t16_tests.log | head -20; exit $rc; }
PREV=$PWD/oac-explore_amd/oac_amd/liboac_amd_prev.so
for r in 1 2; do for v in prev cur; do
  if [ $v = prev ]; then export OAC_LIB=$PREV; else unset OAC_LIB; fi
  timeout -k 10 120 python tools/launch_times.py > gpurun_out/r5_t16_lt_$v.txt 2>&1; rc=$?; crash $rc
  echo "$v: $(grep drop-in gpurun_out/r5_t16_lt_$v.txt | cut -c1-90)"
  grep launch gpurun_out/r5_t16_lt_$v.txt | grep -v drop | awk '{printf "%s ", $4}'; echo
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r5_t16_drv.json 2>/dev/null; rc=$?; crash $rc
  python -c "import json; d=json.loads(open('gpurun_out/r5_t16_drv.json').read().strip().splitlines()[-1]); print('  driver shape', d['value'])"
done; done
