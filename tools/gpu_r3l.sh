#!/bin/bash
# DP drop-in step graph attached to the handle: DP tests, then dp1 vs single
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/dp1_ab.py > gpurun_out/dp1_ab.log 2>&1
rc=$?; tail -c 1500 gpurun_out/dp1_ab.log; exit $rc
