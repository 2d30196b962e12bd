#!/bin/bash
# large-batch kernel loop: parity of every B >= 1024 case, then per-launch timing at B=4096
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_ragged.py tests/test_gpu_goac.py tests/test_gpu_ptrain.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_big.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_big.log; grep -E "^FAILED|Error" gpurun_out/pytest_big.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 300 2>&1 | grep -v amdgpu.ids
