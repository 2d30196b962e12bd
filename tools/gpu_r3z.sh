#!/bin/bash
# critic last-layer dW (+ layer-1 bias at small batch) in the targets kernel: SAC parity suites, then per-launch times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_dropin.py tests/test_gpu_ragged.py tests/test_gpu_altkernels.py tests/test_gpu_ring.py tests/test_gpu_checkpoint.py > gpurun_out/z_tests.log 2>&1 || { tail -40 gpurun_out/z_tests.log; exit 1; }
tail -3 gpurun_out/z_tests.log
timeout -k 10 300 python tools/launch_times.py --batch 256 > gpurun_out/lt_z256.txt 2>&1 &&
timeout -k 10 300 python tools/launch_times.py --batch 4096 > gpurun_out/lt_z4096.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/lt_z256.txt; grep -v amdgpu.ids gpurun_out/lt_z4096.txt
exit $rc
