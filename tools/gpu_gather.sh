#!/bin/bash
# gather copies with loads in flight: drop-in / gather / ring tests, then B=256 and B=4096 per-launch times
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dropin or gather or ring or sac_step or ragged or graph" > gpurun_out/pytest_g.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_g.log; grep -E "^FAILED|Error" gpurun_out/pytest_g.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 20 --rate-steps 3000 > gpurun_out/lt256.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt256.log | tail -14
timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096.log | tail -16 | head -3
