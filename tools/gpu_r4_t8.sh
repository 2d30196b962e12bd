#!/bin/bash
# round 4: the armed single-observation exploration call -- its tests, then
# the per-call wall time armed / plain (OAC_EXPL_ARMED=0) on the same box
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "expl or philox or armed" -v $T > gpurun_out/r4_t8_tests.log 2>&1
rc=$?; crash $rc; grep -E "PASS|FAIL|Error|error" gpurun_out/r4_t8_tests.log | tail -25; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    OAC_EXPL_ARMED=$v timeout -k 10 120 python tools/expl_prof.py --reps 400 > gpurun_out/r4_t8_expl_$v.log 2>&1; crash $?
    echo "armed=$v $(tail -1 gpurun_out/r4_t8_expl_$v.log)"
  done
done
# the row-block dataflow form of the B=256 critic branch against its three launches
timeout -k 10 120 tools/micro/dataflow_micro > gpurun_out/r4_dataflow_micro.log 2>&1; crash $?
cat gpurun_out/r4_dataflow_micro.log
