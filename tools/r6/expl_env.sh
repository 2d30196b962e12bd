#!/bin/bash
# round 6: the exploration call's host wall (tools/micro/expl_micro) under HIP
# runtime settings that move the kernel arguments / the dispatch path
O=$PWD/gpurun_out/r6/explenv
mkdir -p $O
for i in 1 2 3; do
  for v in default "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "AMD_DIRECT_DISPATCH=0"; do
    if [ $v = default ]; then E=""; else E="$v"; fi
    env $E timeout -k 5 60 taskset -c 0-3 tools/micro/expl_micro 400 1 0 > $O/${v}_$i.txt 2>&1 || { echo "expl_micro failed ($v)"; tail -3 $O/${v}_$i.txt; exit 1; }
    echo "$v $i: $(grep -o 'host wall per call [0-9.]* us' $O/${v}_$i.txt)"
  done
done
