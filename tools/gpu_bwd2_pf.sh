#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rollout.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rollout.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_rollout.log; [ $rc -eq 0 ] || exit $rc
for pf in 2 3 4; do
  echo "PF=$pf"; OAC_BWD2_PF=$pf timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 > gpurun_out/lt_pf$pf.txt || exit 1
  grep -E "B=|launch ( 8| 9|11|14|15|16)" gpurun_out/lt_pf$pf.txt
done
