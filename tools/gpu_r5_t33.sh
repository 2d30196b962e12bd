#!/bin/bash
# round 5: where HIP puts the kernel arguments (HIP_FORCE_DEV_KERNARG unset /
# 1 / 0) on the B=256 step -- launch breakdowns and the driver-shaped bench line
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for r in 1 2; do for v in unset 1 0; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 120 python tools/launch_times.py --batch 256 --rate-steps 600 > gpurun_out/r5_t33_b256_$v.txt 2>&1; rc=$?; crash $rc
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r5_t33_bench_$v.txt 2>&1; rc=$?; crash $rc
  echo "kernarg $v | $(grep drop-in gpurun_out/r5_t33_b256_$v.txt | cut -c1-70) | bench20 $(tail -1 gpurun_out/r5_t33_bench_$v.txt | grep -o '"value": [0-9.]*')"
done; done
