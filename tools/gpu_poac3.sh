#!/bin/bash
# P-OAC: dh2 of the K-output head in the targets kernel (OAC_DH2_TARGETS)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "particle or poac or dp or checkpoint or dropin" > gpurun_out/pytest_poac.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_poac.log; grep -E "^FAILED|Error" gpurun_out/pytest_poac.log | head; [ $rc -eq 0 ] || exit $rc
for v in "OAC_DH2_TARGETS=1"; do
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/ltp_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v "^launch" gpurun_out/ltp_$v.log | tail -19 | sed -n '1p;6,9p'
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 256 --steps 10 --rate-steps 2000 > gpurun_out/ltp256_$v.log 2>&1 || exit $?
  grep "drop-in" gpurun_out/ltp256_$v.log
done
