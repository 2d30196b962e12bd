#!/bin/bash
# rank-R epilogue operands prefetched before the k loop: GPU tests, then B=256 / B=4096 rates
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_all.log; grep -E "^FAILED|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 20 --rate-steps 4000 > gpurun_out/lt256.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt256.log | tail -13 | head -3
timeout -k 5 120 python tools/launch_times.py --poac --batch 256 --steps 20 --rate-steps 2000 > gpurun_out/ltp256.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/ltp256.log | tail -20 | head -1
