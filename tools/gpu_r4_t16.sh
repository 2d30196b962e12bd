#!/bin/bash
# round 4 A/B at B=256: the -min Q backward merged into the critic layer-0 dW
# launch (OAC_MINQ_MERGE) and that launch's obs-column dW deferred to the
# policy-backward launches (OAC_DW0_DEFER); parity first
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_teacher.py tests/test_gpu_ring.py tests/test_gpu_checkpoint.py tests/test_gpu_ragged.py -q -x $T > gpurun_out/r4_t16_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r4_t16_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    OAC_MINQ_MERGE=$1 OAC_DW0_DEFER=$2 timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t16_lt_$1$2.log 2>&1; crash $?
    echo "merge=$1 defer=$2 $(grep drop-in gpurun_out/r4_t16_lt_$1$2.log)"
  done
done
grep 'launch ' gpurun_out/r4_t16_lt_11.log | tr -s ' ' | tr '\n' '|'; echo
