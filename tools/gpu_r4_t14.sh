#!/bin/bash
# small-kernel stage clocks (gemm_micro, -DOAC_STAGE_CLOCK) and the launch floor
mkdir -p gpurun_out
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro.log 2>&1 || exit 1
timeout -k 10 120 tools/micro/floor_micro > gpurun_out/r4_floor_micro.log 2>&1 || exit 1
grep -v "gpw [346]" gpurun_out/r4_gemm_micro.log
