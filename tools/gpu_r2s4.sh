#!/bin/bash
# session-4 baseline: head micro at B=4096 and per-launch times (SAC B=4096, configs[4])
mkdir -p gpurun_out
for cc in 2 4 8; do timeout -k 5 60 tools/micro/head_micro 4096 $cc || exit $?; done
OAC_DEBUG_CFG=1 timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 300 > gpurun_out/lt4096.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096.log | tail -24
OAC_DEBUG_CFG=1 timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 300 > gpurun_out/lt_poac.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt_poac.log | tail -24
