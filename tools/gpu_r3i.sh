#!/bin/bash
# B=4096 direct gather (row-indexed LDS-DMA forward + side copy blocks): the
# GPU suite, then per-launch times and the drop-in rate at B=4096 and B=256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputest_r3i.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 8 --rate-steps 1000 > gpurun_out/lt4096.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 256 --steps 20 --rate-steps 3000 > gpurun_out/lt256.log 2>&1
rc=$?
tail -2 gpurun_out/gputest_r3i.log; cat gpurun_out/lt4096.log gpurun_out/lt256.log
exit $rc
