#!/bin/bash
# A/B of the B=256 drop-in step: OAC_SMALL_STAGE=0 / 1 (small-kernel operands
# staged through LDS by LDS-DMA), alternated, 3 runs each; per-launch times of both
mkdir -p gpurun_out
for i in 1 2 3; do
  for st in 0 1; do
    OAC_SMALL_STAGE=$st timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/ab_stage_$st.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_stage_$st.log').read().strip().splitlines()[-1]);print('stage=$st', d['value'], d['roofline']['avg_launch_us'])"
  done
done
for st in 0 1; do
  OAC_SMALL_STAGE=$st timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_stage_$st.log 2>&1 || exit 1
  head -14 gpurun_out/lt_stage_$st.log
done
