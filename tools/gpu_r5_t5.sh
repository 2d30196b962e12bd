#!/bin/bash
# round 5: the LDS-transposed vector-store epilogue of the pipelined GEMMs --
# micro outputs vs the register-direct kernel, clocks, same-box A/B, parity
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 120 tools/micro/bwd_micro 12 3 > gpurun_out/r5_t5_bwd.txt 2>&1; rc=$?; crash $rc; cat gpurun_out/r5_t5_bwd.txt
timeout -k 10 120 tools/micro/fwd_micro > gpurun_out/r5_t5_fwd.txt 2>&1; rc=$?; crash $rc; cat gpurun_out/r5_t5_fwd.txt | tail -8
timeout -k 10 120 tools/micro/bwd_clock_micro 12 12 > gpurun_out/r5_t5_bwdclk.txt 2>&1; rc=$?; crash $rc; grep clocks gpurun_out/r5_t5_bwdclk.txt
timeout -k 10 120 tools/micro/fwd_clock_micro > gpurun_out/r5_t5_fwdclk.txt 2>&1; rc=$?; crash $rc; grep clocks gpurun_out/r5_t5_fwdclk.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_altkernels.py tests/test_gpu_teacher.py tests/test_gpu_ragged.py tests/test_gpu_goac.py tests/test_gpu_ptrain.py -q -x $T > gpurun_out/r5_t5_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 bash tools/ab_lib.sh 4096; rc=$?; crash $rc
timeout -k 10 500 bash tools/ab_lib.sh 4096 --poac; rc=$?; crash $rc
