#!/bin/bash
# small-batch critic layers one launch later (OAC_REBAL): GPU tests, then B=256 A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_REBAL=1" "OAC_REBAL=0" "OAC_REBAL=1" "OAC_REBAL=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 20 --rate-steps 4000 > gpurun_out/ltr_$v.log 2>&1 || exit $?
  echo "$v: $(grep drop-in gpurun_out/ltr_$v.log) $(grep 'launch  0\|launch  1 \|launch  3 ' gpurun_out/ltr_$v.log | tr -s ' ' | tr '\n' ' ')"
done
