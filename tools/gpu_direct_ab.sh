#!/bin/bash
mkdir -p gpurun_out
for v in "OAC_DROPIN_DIRECT=1" "OAC_DROPIN_DIRECT=0" "OAC_DROPIN_DIRECT=1" "OAC_DROPIN_DIRECT=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 10 --rate-steps 4000 > gpurun_out/ltd_$v.log 2>&1 || exit $?
  echo "$v: $(grep drop-in gpurun_out/ltd_$v.log) $(grep 'launch  0\|launch  1 ' gpurun_out/ltd_$v.log | tr -s ' ' | tr '\n' ' ')"
done
for v in "OAC_HOSTIDX=1" "OAC_HOSTIDX=0"; do
  env $v timeout -k 5 120 python tools/launch_times.py --poac --batch 256 --steps 10 --rate-steps 2000 > gpurun_out/ltdp_$v.log 2>&1 || exit $?
  echo "poac $v: $(grep drop-in gpurun_out/ltdp_$v.log)"
done
