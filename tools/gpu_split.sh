#!/bin/bash
# side-workgroup Adam (OAC_SPLIT_ADAM) + one-chunk head: GPU tests, then B=4096 per-launch times A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log; grep -E "FAIL|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_SPLIT_ADAM=0" "OAC_SPLIT_ADAM=1" "OAC_SIDE_BLOCKS=64" "OAC_SIDE_BLOCKS=128"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 400 > gpurun_out/lt_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/lt_$v.log | tail -17
done
