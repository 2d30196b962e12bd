#!/bin/bash
# large-batch GPU tests + per-launch times at B=4096 (one pytest process)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${K:-b4096 or ragged or particle or goac or ptrain or dp or big or 1024}" > gpurun_out/pytest_big.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_big.log; [ $rc -eq 0 ] || exit $rc
OAC_DEBUG_CFG=1 timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 200 > gpurun_out/lt4096.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096.log | tail -18
