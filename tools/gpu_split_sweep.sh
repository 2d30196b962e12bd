#!/bin/bash
# B=4096 drop-in rate over split-K settings (same box)
mkdir -p gpurun_out
run() { echo "$1: $(env $1 timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 | head -1 | cut -c1-60)"; }
run "OAC_NONE=1" || exit 1
run "OAC_SPLIT_KMIN=256" || exit 1
run "OAC_SPLIT_KMIN=512" || exit 1
run "OAC_SPLITS=8,8,8,8,8" || exit 1
run "OAC_SPLITS=12,12,8,12,12" || exit 1
run "OAC_SPLITS=24,24,16,24,24" || exit 1
run "OAC_NONE=2" || exit 1
