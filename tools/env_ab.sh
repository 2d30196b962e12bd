#!/bin/bash
# A/B of runtime environment switches on the B=256 drop-in step
mkdir -p gpurun_out
for env in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "X=0"; do
  env $env timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
  echo "$env $(python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_launch_us'], d['kernels']['row']['avg_us'])")"
done
