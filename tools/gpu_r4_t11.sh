#!/bin/bash
# round 4 A/B: multi-step graph launches (ring path, counts recipes) against
# direct launches (OAC_STEP_GRAPH=0), the bench's extras legs
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for v in 1 0; do
    OAC_STEP_GRAPH=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4_t11_$v.log 2>&1; crash $?
    python -c "
import json;d=json.loads(open('gpurun_out/r4_t11_$v.log').read().strip().splitlines()[-1])
print('graph=$v', 'b256', d['value'], 'ring', d['ring']['steps_per_s'], 'goac', d['goac']['steps_per_s'], 'poac256', d['poac']['steps_per_s'], 'dp1', d['dp1']['steps_per_s'], 'b4096', d['b4096']['steps_per_s'], 'cfg4', d['poac_ant_b4096']['steps_per_s'])"
  done
done
