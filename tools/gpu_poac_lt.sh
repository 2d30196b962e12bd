#!/bin/bash
# per-launch times of configs[4] (P-OAC K=10, Ant dims, B=4096) with launch configs
mkdir -p gpurun_out
OAC_DEBUG_CFG=1 timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 300 > gpurun_out/lt_poac.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt_poac.log | tail -24
grep "^launch" gpurun_out/lt_poac.log | head -22 | cut -c1-220
