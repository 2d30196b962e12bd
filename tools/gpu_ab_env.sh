#!/bin/bash
# same-box A/B of an env switch on the B=4096 SAC and configs[4] P-OAC drop-in rates:
#   VAR=OAC_NARROWM_SMALL A=0 B=1 bash tools/gpu_ab_env.sh
mkdir -p gpurun_out
for v in $A $B $A $B; do
  echo "== $VAR=$v"
  env $VAR=$v timeout -k 5 100 python tools/launch_times.py --batch 4096 --steps 5 --rate-steps 400 2>&1 | grep drop-in || exit 1
  env $VAR=$v timeout -k 5 100 python tools/launch_times.py --poac --batch 4096 --steps 5 --rate-steps 400 2>&1 | grep drop-in || exit 1
done 2>&1 | tee gpurun_out/ab_env.log
