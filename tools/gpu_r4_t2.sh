#!/bin/bash
# round 4: new tests + GPU suite + bench, then the small-GEMM launch micro and TA counters
mkdir -p gpurun_out
bash tools/gpu_r4_t1.sh || exit $?
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro.log 2>&1 || exit 1
timeout -k 10 60 tools/micro/floor_micro > gpurun_out/r4_floor_micro.log 2>&1 || exit 1
bash tools/pmc_ta.sh b256
head -5 gpurun_out/r4_gemm_micro.log
