#!/bin/bash
# host-read index ring (no H2D copy before the drop-in step): full GPU tests, then A/B step rates
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_HOSTIDX=1" "OAC_HOSTIDX=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lth_$v.log 2>&1 || exit $?
  echo "== sac $v: $(grep drop-in gpurun_out/lth_$v.log)"
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lthp_$v.log 2>&1 || exit $?
  echo "== poac $v: $(grep drop-in gpurun_out/lthp_$v.log)"
done
