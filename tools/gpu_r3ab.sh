#!/bin/bash
# launch geometry (cfg, workgroups, tasks) of the B=4096 SAC and configs[4] P-OAC steps
set -o pipefail
mkdir -p gpurun_out
OAC_DEBUG_CFG=1 timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 2 --rate-steps 4 > gpurun_out/cfg_sac.txt 2>&1 &&
OAC_DEBUG_CFG=1 timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 --steps 2 --rate-steps 4 > gpurun_out/cfg_poac.txt 2>&1
rc=$?
grep "^launch" gpurun_out/cfg_sac.txt | sort | uniq -c | sort -k3 -n | head -30
echo ---
grep "^launch" gpurun_out/cfg_poac.txt | sort | uniq -c | sort -k3 -n | head -30
exit $rc
