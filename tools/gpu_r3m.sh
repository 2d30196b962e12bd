#!/bin/bash
# where the time goes: exploration stage clocks, launch floor, per-launch
# breakdowns of the B=4096 SAC step and configs[4]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/expl_micro 400 1 > gpurun_out/expl_micro.log 2>&1 &&
timeout -k 10 60 tools/micro/launch_wall_micro > gpurun_out/launch_wall.log 2>&1 &&
timeout -k 10 200 python tools/launch_times.py --batch 4096 > gpurun_out/lt_b4096.log 2>&1 &&
timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/lt_poac.log 2>&1 &&
timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_b256.log 2>&1
rc=$?
tail -n 30 gpurun_out/expl_micro.log gpurun_out/launch_wall.log
tail -n 22 gpurun_out/lt_b4096.log gpurun_out/lt_poac.log gpurun_out/lt_b256.log
exit $rc
