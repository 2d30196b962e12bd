#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 20 --rate-steps 4000 > gpurun_out/lts_$i.log 2>&1 || exit $?
  echo "$(grep drop-in gpurun_out/lts_$i.log) $(grep 'launch  4' gpurun_out/lts_$i.log)"
done
