#!/bin/bash
# the backward micro-benchmark with device launch records (OAC_MICRO_DEVREC,
# the plans' form) against by-value records, two builds interleaved
O=$PWD/gpurun_out/r6/devrec
mkdir -p $O
for r in 1 2; do for v in $VARIANTS; do for d in 0 1; do
  if [ $d = 1 ]; then export OAC_MICRO_DEVREC=1; else unset OAC_MICRO_DEVREC; fi
  LD_LIBRARY_PATH=$PWD/tools/r6/libs/$v timeout -k 5 60 tools/micro/bwd_micro 12 1 > $O/${v}_$d_$r.txt 2>&1 || exit $?
  echo "$v devrec=$d r$r: $(sed 's/.*cfg12 *//' $O/${v}_$d_$r.txt | awk '{printf "%s ", $1}')"
done; done; done
