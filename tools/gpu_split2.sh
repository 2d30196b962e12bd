#!/bin/bash
# side-workgroup Adam placement / count A/B at B=4096 (SAC, configs[4]), then the large-batch tests
mkdir -p gpurun_out
for v in "OAC_SIDE_FIRST=1" "OAC_SIDE_FIRST=0" "OAC_SIDE_BLOCKS=256" "OAC_SPLIT_ADAM=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 400 > gpurun_out/lt_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/lt_$v.log | tail -17 | sed -n '1p;8,15p'
done
for v in "OAC_SPLIT_ADAM=1" "OAC_SPLIT_ADAM=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 400 > gpurun_out/ltp_$v.log 2>&1 || exit $?
  echo "== poac $v"; grep -v "^launch" gpurun_out/ltp_$v.log | tail -24 | sed -n '1p;10,13p;19,24p'
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "b4096 or ragged or 1024 or dropin or checkpoint or particle or poac" > gpurun_out/pytest_big.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_big.log; exit $rc
