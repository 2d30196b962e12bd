#!/bin/bash
# round 4 A/B: the drop-in step as one graph launch (default) or as direct
# launches (OAC_DROPIN_DIRECT=1), B=256 bench line and B=4096 / configs[4]
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for v in 0 1; do
    OAC_DROPIN_DIRECT=$v timeout -k 10 200 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/r4_t9_b256_$v.log 2>&1; crash $?
    python -c "import json;d=json.loads(open('gpurun_out/r4_t9_b256_$v.log').read().strip().splitlines()[-1]);print('direct=$v B=256', d['value'], d['ms_per_step'])"
    OAC_DROPIN_DIRECT=$v timeout -k 10 200 python tools/launch_times.py --batch 4096 > gpurun_out/r4_t9_lt.log 2>&1; crash $?
    echo "direct=$v $(grep -v amdgpu gpurun_out/r4_t9_lt.log | head -1)"
    OAC_DROPIN_DIRECT=$v timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/r4_t9_lt.log 2>&1; crash $?
    echo "direct=$v poac $(grep -v amdgpu gpurun_out/r4_t9_lt.log | head -1)"
  done
done
# the dataflow critic branch with its batches in the kernel arguments (global loads)
timeout -k 10 120 tools/micro/dataflow_micro > gpurun_out/r4_dataflow_micro2.log 2>&1; crash $?
cat gpurun_out/r4_dataflow_micro2.log
