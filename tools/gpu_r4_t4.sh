#!/bin/bash
# round 4: micros, TA counters, the full GPU suite (defaults)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro.log 2>&1; crash $?
bash tools/pmc_ta.sh b256
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_all.log 2>&1
rc=$?; tail -5 gpurun_out/r4_pytest_all.log; exit $rc
