#!/bin/bash
# side-branch critic layer 1 (OAC_FORK): GPU tests, then A/B step rates
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_FORK=1" "OAC_FORK=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 4 --rate-steps 600 > gpurun_out/ltf_$v.log 2>&1 || exit $?
  echo "== sac4096 $v: $(grep drop-in gpurun_out/ltf_$v.log)"
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 4 --rate-steps 600 > gpurun_out/ltfp_$v.log 2>&1 || exit $?
  echo "== poac4096 $v: $(grep drop-in gpurun_out/ltfp_$v.log)"
  env $v timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 4 --rate-steps 4000 > gpurun_out/ltf256_$v.log 2>&1 || exit $?
  echo "== sac256 $v: $(grep drop-in gpurun_out/ltf256_$v.log)"
done
