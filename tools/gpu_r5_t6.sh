#!/bin/bash
# round 5: P-OAC row kernels -- the NaN-safe rank sort as integer keys and the
# argmin row by value selects, against the round-4 kernels (same box)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_particle.py tests/test_gpu_ptrain.py tests/test_gpu_teacher.py -q -x $T -k "particle or ptrain or poac" > gpurun_out/r5_t6_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r5_t6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab_lib.sh 4096 --poac; rc=$?; crash $rc
