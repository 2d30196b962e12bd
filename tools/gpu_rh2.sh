#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "particle or poac or dp or goac or ptrain" > gpurun_out/pytest_poac.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_poac.log; grep -E "^FAILED|Error" gpurun_out/pytest_poac.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/ltp.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/ltp.log | tail -19 | sed -n '1p;7p'
timeout -k 5 120 python tools/launch_times.py --poac --batch 256 --steps 10 --rate-steps 2000 > gpurun_out/ltp256.log 2>&1 || exit $?
grep "drop-in" gpurun_out/ltp256.log
