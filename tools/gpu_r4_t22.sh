#!/bin/bash
# round 4: the deferred critic layer-0 Adam (preview into the shadow, side
# blocks in the policy-head launch) after cleanup; parity + ring split first
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_teacher.py tests/test_gpu_ring.py tests/test_gpu_checkpoint.py -q -x $T > gpurun_out/r4_t22_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r4_t22_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    OAC_DW0_DEFER=$v timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t22_lt_$v.log 2>&1; crash $?
    echo "defer=$v $(grep drop-in gpurun_out/r4_t22_lt_$v.log)"
  done
done
grep 'launch ' gpurun_out/r4_t22_lt_1.log | tr -s ' ' | tr '\n' '|'; echo
