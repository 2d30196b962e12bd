#!/bin/bash
# full GPU suite, the backward micro-benchmark, then per-launch times at
# B=4096 (SAC and configs[4]) and B=256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 60 tools/micro/bwd_micro 10 > gpurun_out/bwd_micro.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ltpoac.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 256 --steps 40 --rate-steps 4000 > gpurun_out/lt256.log 2>&1
rc=$?
tail -3 gpurun_out/gputest.log; cat gpurun_out/bwd_micro.log gpurun_out/lt4096.log gpurun_out/ltpoac.log gpurun_out/lt256.log | grep -v amdgpu.ids
exit $rc
