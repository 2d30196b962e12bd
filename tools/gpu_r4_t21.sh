#!/bin/bash
# the full GPU suite after the Adam / Polyak contraction fix, then the
# OAC_DW0_DEFER 1 / 2 A/B at B=256
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t21_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r4_t21_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 2; do
    OAC_DW0_DEFER=$v timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t21_lt_$v.log 2>&1; crash $?
    echo "defer=$v $(grep drop-in gpurun_out/r4_t21_lt_$v.log)"
  done
done
