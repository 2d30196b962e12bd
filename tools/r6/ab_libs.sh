#!/bin/bash
# round 6: same-box interleaved A/B of library builds (tools/r6/libs/<name>/
# liboac_amd.so): the backward micro-benchmark (bwd_micro, LD_LIBRARY_PATH)
# and the step's per-launch durations + rate at B=4096 SAC and configs[4]
# (tools/launch_times.py, OAC_LIB).  VARIANTS="base lb4 ..."; ROUNDS (2);
# LEGS (micro b4096 poac b256)
R=$PWD
O=$R/gpurun_out/r6/${TAG:-ab}
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
LEGS=${LEGS:-micro b4096 poac}
for r in $(seq 1 ${ROUNDS:-2}); do
for v in $VARIANTS; do
  L=$R/tools/r6/libs/$v/liboac_amd.so
  for leg in $LEGS; do
    case $leg in
      micro) LD_LIBRARY_PATH=$R/tools/r6/libs/$v timeout -k 5 60 tools/micro/bwd_micro ${CFG:-12} 1 > $O/${v}_micro_$r.txt 2>&1; crash $?
             echo "$v micro r$r: $(awk '{printf "%s ", $(NF-6)}' $O/${v}_micro_$r.txt)";;
      b4096) OAC_LIB=$L timeout -k 10 150 python tools/launch_times.py --batch 4096 --rate-steps 600 > $O/${v}_b4096_$r.txt 2>&1; crash $?
             echo "$v b4096 r$r: $(grep drop-in $O/${v}_b4096_$r.txt | cut -c1-100)"
             grep "launch " $O/${v}_b4096_$r.txt | awk '{printf "%s ", $4}'; echo;;
      poac)  OAC_LIB=$L timeout -k 10 150 python tools/launch_times.py --batch 4096 --poac --rate-steps 600 > $O/${v}_poac_$r.txt 2>&1; crash $?
             echo "$v poac r$r: $(grep drop-in $O/${v}_poac_$r.txt | cut -c1-100)"
             grep "launch " $O/${v}_poac_$r.txt | awk '{printf "%s ", $4}'; echo;;
      b256)  OAC_LIB=$L timeout -k 10 150 python tools/launch_times.py --rate-steps 2000 > $O/${v}_b256_$r.txt 2>&1; crash $?
             echo "$v b256 r$r: $(grep drop-in $O/${v}_b256_$r.txt | cut -c1-100)";;
    esac
  done
done; done
