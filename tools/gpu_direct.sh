#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_direct.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_direct.log; grep -E "^FAILED|Error" gpurun_out/pytest_direct.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_direct.txt || exit 1
cat gpurun_out/lt_direct.txt
OAC_DROPIN_DIRECT=0 timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_nodirect.txt || exit 1
head -1 gpurun_out/lt_nodirect.txt
