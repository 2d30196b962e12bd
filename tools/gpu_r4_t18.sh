#!/bin/bash
# small-kernel stage clocks incl. a fused-Adam dW batch (gemm_micro)
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro2.log 2>&1 || exit 1
grep -A1 "nw  0" gpurun_out/r4_gemm_micro2.log
