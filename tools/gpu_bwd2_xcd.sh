#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "4096 or b4096 or dp or poac or particle or goac" > gpurun_out/pytest_xcd.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_xcd.log; grep -E "^FAILED" gpurun_out/pytest_xcd.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 > gpurun_out/lt_xcd.txt || exit 1
cat gpurun_out/lt_xcd.txt
