#!/bin/bash
# same-box A/B of two library builds: tools/ab_lib.sh <batch> [--poac] (base = oac_amd/liboac_amd_base.so)
B=${1:-4096}; shift
mkdir -p gpurun_out
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export OAC_LIB=$PWD/oac-explore_amd/oac_amd/liboac_amd_base.so; else unset OAC_LIB; fi
    timeout -k 10 200 python tools/launch_times.py --batch $B --rate-steps 500 "$@" > gpurun_out/ab_${v}_$r.txt || exit 1
    echo "$v run $r: $(head -1 gpurun_out/ab_${v}_$r.txt)"
  done
done
paste gpurun_out/ab_base_2.txt gpurun_out/ab_new_2.txt | tail -n +2 | awk '{printf "%s %s %s | %s\n", $2, $3, $4, $9}'
