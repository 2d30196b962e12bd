#!/bin/bash
# cfg-5 backward kernel: GPU tests, then per-launch times at B=4096 with and without it
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_bwd2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_bwd2.log; grep -E "^FAILED|Error" gpurun_out/pytest_bwd2.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 || exit 1
OAC_BWD2=0 timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 | head -1
