#!/bin/bash
# round 4 (after removing the B=256 A/B variants): the teacher-forced and
# drop-in tests (incl. the direct large-batch gather cases), the exploration
# micro, and configs[4] with / without the direct gather (A/B, same box)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_dropin.py tests/test_gpu_ring.py -v $T -s > gpurun_out/r4_t5_tests.log 2>&1
rc=$?; crash $rc; grep -E "PASS|FAIL|b4096 step|Error" gpurun_out/r4_t5_tests.log | cut -c1-400 | tail -40; echo "tests rc=$rc"
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/r4_expl_micro.log 2>&1; crash $?
head -16 gpurun_out/r4_expl_micro.log
for i in 1 2; do
  for d in 1 0; do
    OAC_POAC_DIRECT=$d timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/lt_poac_d$d.log 2>&1
    crash $?; echo "direct=$d"; grep -v amdgpu gpurun_out/lt_poac_d$d.log | head -1
  done
done
grep -v amdgpu gpurun_out/lt_poac_d1.log | head -20
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4_t5_bench.log 2>&1; crash $?
tail -1 gpurun_out/r4_t5_bench.log | cut -c1-400
