#!/bin/bash
# round 6: the last-arrival policy layer-0 Adam (tuning la_adam) -- the
# bitwise / oracle tests, then interleaved step A/B (B=4096 SAC) against the
# Adam launch
O=$PWD/gpurun_out/r6/${TAG:-la}
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_altkernels.py -k "last_arrival or side_workgroup" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
grep -E "PASS|FAIL" $O/tests.txt | cut -c1-150
for r in 1 2 3; do
  for la in 0 1; do
    OAC_TUNE=la_adam=$la timeout -k 10 150 python tools/launch_times.py --batch 4096 --rate-steps 600 > $O/s_${la}_$r.txt 2>&1; crash $?
    echo "b4096 la=$la r$r: $(grep drop-in $O/s_${la}_$r.txt | cut -c1-70)"
    grep "launch " $O/s_${la}_$r.txt | awk '{printf "%s ", $4}'; echo
  done
done
