#!/bin/bash
# round 4 A/B: the -min Q backward inside the critic layer-0 dW launch
# (OAC_MINQ_MERGE=1, default; 0 = its own launch), parity first
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_teacher.py tests/test_gpu_ring.py tests/test_gpu_checkpoint.py tests/test_gpu_ragged.py -q -x $T > gpurun_out/r4_t15_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r4_t15_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 0 1; do
    OAC_MINQ_MERGE=$v timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t15_lt_$v.log 2>&1; crash $?
    echo "merge=$v $(grep drop-in gpurun_out/r4_t15_lt_$v.log)"
  done
done
grep 'launch ' gpurun_out/r4_t15_lt_1.log | tr -s ' ' | tr '\n' '|'; echo
