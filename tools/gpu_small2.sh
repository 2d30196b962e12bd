#!/bin/bash
# small kernel with unconditional k-loop loads: GPU tests, B=256 / P-OAC / B=4096 rates
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 10 --rate-steps 4000 > gpurun_out/lt256.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt256.log | tail -13
timeout -k 5 120 python tools/launch_times.py --poac --batch 256 --steps 10 --rate-steps 2000 > gpurun_out/ltp256.log 2>&1 || exit $?
grep "drop-in" gpurun_out/ltp256.log
timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 || exit $?
grep "drop-in" gpurun_out/lt4096.log
