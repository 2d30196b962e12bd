#!/bin/bash
# exploration group-size sweep (twin kernel), then the suite and launch times
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/expl_group.log
for g in 32 16 24 32 16 24 8; do
  timeout -k 10 60 tools/micro/expl_micro 400 1 0 $g | head -1 >> gpurun_out/expl_group.log || exit 1
done
cat gpurun_out/expl_group.log
bash tools/gpu_r3p.sh
