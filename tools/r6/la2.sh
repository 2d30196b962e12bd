#!/bin/bash
# round 6: last-arrival Adam with the policy layer-0 dW split fewer ways
O=$PWD/gpurun_out/r6/${TAG:-la3}
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2; do
  for spec in "la_adam=0" "la_adam=1" "la_adam=1,splits_p0=8"; do
    tag=$(echo $spec | tr ',=' '__')
    OAC_TUNE=$spec timeout -k 10 150 python tools/launch_times.py --batch 4096 --rate-steps 600 > $O/s_${tag}_$r.txt 2>&1; crash $?
    echo "b4096 $spec r$r: $(grep drop-in $O/s_${tag}_$r.txt | cut -c1-70)"
    grep "launch " $O/s_${tag}_$r.txt | awk '{printf "%s ", $4}'; echo
  done
done
