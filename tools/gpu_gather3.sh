#!/bin/bash
# gather kernel change: the gather-path tests, then per-launch times at B=4096
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_ragged.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gather_tests.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ltpoac.log 2>&1
rc=$?
tail -2 gpurun_out/gather_tests.log; cat gpurun_out/lt4096.log gpurun_out/ltpoac.log | grep -v amdgpu.ids
exit $rc
