#!/bin/bash
# threshold sweep of the small-forward-batch tile choice (B=4096 SAC and configs[4] P-OAC)
mkdir -p gpurun_out
for v in 256 512 1024; do
  echo "OAC_SMALL_FWD=$v poac: $(OAC_SMALL_FWD=$v timeout -k 10 300 python tools/launch_times.py --poac --batch 4096 --rate-steps 300 --steps 10 | head -1 | cut -c1-60)"
  echo "OAC_SMALL_FWD=$v sac:  $(OAC_SMALL_FWD=$v timeout -k 10 300 python tools/launch_times.py --batch 4096 --rate-steps 300 --steps 10 | head -1 | cut -c1-60)"
done
