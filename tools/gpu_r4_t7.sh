#!/bin/bash
# round 4: P-OAC row kernels with the backward operands prefetched (targets,
# min) and the alpha update on its own block -- parity then per-launch times
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_particle.py tests/test_gpu_teacher.py tests/test_gpu_ring.py tests/test_gpu_dropin.py tests/test_gpu_dp.py -q -x $T > gpurun_out/r4_t7_tests.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r4_t7_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/lt_t7.log 2>&1; crash $?
  grep -v amdgpu gpurun_out/lt_t7.log | head -18
done
