#!/bin/bash
# A/B of the B=256 drop-in step: OAC_SMALL_STAGE=0 / 1 (small-kernel operands
# staged through LDS by LDS-DMA), alternated, 3 runs each; per-launch times of both
mkdir -p gpurun_out
# arms: "stage pbwd" = OAC_SMALL_STAGE, OAC_PBWD_FUSE
for i in 1 2 3; do
  for arm in "0 0" "1 0" "0 1" "1 1"; do
    set -- $arm
    OAC_SMALL_STAGE=$1 OAC_PBWD_FUSE=$2 timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/ab_s$1_p$2.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_s$1_p$2.log').read().strip().splitlines()[-1]);print('stage=$1 pbwd=$2', d['value'], d['roofline']['avg_launch_us'], d['roofline']['launches_per_step'])"
  done
done
for arm in "0 0" "1 0" "0 1" "1 1"; do
  set -- $arm
  OAC_SMALL_STAGE=$1 OAC_PBWD_FUSE=$2 timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_s$1_p$2.log 2>&1 || exit 1
  echo "stage=$1 pbwd=$2"; head -16 gpurun_out/lt_s$1_p$2.log
done
