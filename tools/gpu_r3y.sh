#!/bin/bash
# last-layer dW slabs in the targets kernel: large-batch parity (SAC goldens, DP, ragged, alt kernels), then B=4096 per-launch times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_dropin.py tests/test_gpu_ragged.py tests/test_gpu_altkernels.py tests/test_gpu_ring.py > gpurun_out/y_tests.log 2>&1 || { tail -40 gpurun_out/y_tests.log; exit 1; }
tail -3 gpurun_out/y_tests.log
timeout -k 10 300 python tools/launch_times.py --batch 4096 > gpurun_out/lt_y.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/lt_y.txt
exit $rc
