#!/bin/bash
# configs[4] forward-tile sweep (every forward launch forced to one tile / ring depth)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/poac_fwd_sweep.txt
for E in "X=0" "OAC_FWD2_TILE=64,64" "OAC_FWD2_TILE=128,128" "OAC_FWD2_NB=2"; do
  env $E timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 > gpurun_out/pf.txt 2>&1 || { cat gpurun_out/pf.txt; exit 1; }
  echo "$E" >> gpurun_out/poac_fwd_sweep.txt
  grep -v amdgpu.ids gpurun_out/pf.txt >> gpurun_out/poac_fwd_sweep.txt
done
grep -E "^X=|^OAC|drop-in" gpurun_out/poac_fwd_sweep.txt
