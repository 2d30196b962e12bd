#!/bin/bash
# the N-rank bench path rehearsed on one GPU (2 ranks, gloo, same device)
set -o pipefail
mkdir -p gpurun_out
OAC_BENCH_SAME_DEVICE=1 OAC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 64 --warmup 16 --no-cpu-baseline > gpurun_out/bench_n2_gloo.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/bench_n2_gloo.log | tail -c 1500
exit $rc
