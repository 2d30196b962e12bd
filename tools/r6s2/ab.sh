#!/bin/bash
# Same-box A/B of tuning specs on the B=256 per-launch times and drop-in rate:
# tools/r6s2/ab.sh "spec1" "spec2" ... (empty string = default), two rounds.
O=$PWD/gpurun_out/r7
mkdir -p $O
TAG=${TAG:-ab}
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for round in 1 2; do
  for spec in "$@"; do
    echo "== round $round spec '$spec'" >> $O/ab_$TAG.txt
    OAC_TUNE="$spec" timeout -k 10 200 python tools/launch_times.py --batch ${B:-256} >> $O/ab_$TAG.txt 2>&1; crash $?
  done
done
grep -E "==|drop-in|launch  7" $O/ab_$TAG.txt
