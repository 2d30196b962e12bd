#!/bin/bash
# round 4 A/B: multi-step graph launches (ring path, counts recipes) against
# direct launches (OAC_STEP_GRAPH=0), the bench's extras legs
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
# (first: the P-OAC tests after the targets kernel's rank sort)
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_gpu_particle.py tests/test_gpu_teacher.py tests/test_gpu_ring.py -q -x $T > gpurun_out/r4_t11_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r4_t11_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/r4_t11_lt.log 2>&1; crash $?
grep -v amdgpu gpurun_out/r4_t11_lt.log | head -7
for i in 1 2; do
  for v in 1 0; do
    OAC_STEP_GRAPH=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4_t11_$v.log 2>&1; crash $?
    python -c "
import json;d=json.loads(open('gpurun_out/r4_t11_$v.log').read().strip().splitlines()[-1])
print('graph=$v', 'b256', d['value'], 'ring', d['ring']['steps_per_s'], 'goac', d['goac']['steps_per_s'], 'poac256', d['poac']['steps_per_s'], 'dp1', d['dp1']['steps_per_s'], 'b4096', d['b4096']['steps_per_s'], 'cfg4', d['poac_ant_b4096']['steps_per_s'])"
  done
done
