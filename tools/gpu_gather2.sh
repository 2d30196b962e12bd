#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gather or ring or dropin or b4096 or particle or goac" > gpurun_out/pytest_g.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_g.log; grep -E "^FAILED|Error" gpurun_out/pytest_g.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_GATHER_FLAT=1" "OAC_GATHER_FLAT=0" "OAC_GATHER_FLAT=1"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lt4096_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/lt4096_$v.log | tail -16 | head -2
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/ltp4096_$v.log 2>&1 || exit $?
  grep -v "^launch" gpurun_out/ltp4096_$v.log | tail -21 | head -2
done
