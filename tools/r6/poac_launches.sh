#!/bin/bash
# the configs[4] step's GEMM launches (tuning debug_cfg) and per-launch times
O=$PWD/gpurun_out/r6
mkdir -p $O
OAC_TUNE=debug_cfg=1 timeout -k 10 150 python tools/launch_times.py --batch 4096 --poac --rate-steps 50 --steps 2 > $O/poac_launches.txt 2> $O/poac_launches_cfg.txt
rc=$?
sort $O/poac_launches_cfg.txt | uniq -c | sort -k2 | head -40
exit $rc
