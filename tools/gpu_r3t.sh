#!/bin/bash
# particle row kernels with prefetched backward operands: P-OAC / p-oac parity, then configs[4] per-launch times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_particle.py tests/test_gpu_ptrain.py tests/test_gpu_parity.py tests/test_gpu_ragged.py > gpurun_out/r3t_tests.log 2>&1 || { tail -30 gpurun_out/r3t_tests.log; exit 1; }
tail -3 gpurun_out/r3t_tests.log
timeout -k 10 300 python tools/launch_times.py --poac --batch 4096 > gpurun_out/r3t_poac.txt 2>&1 || { tail -20 gpurun_out/r3t_poac.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3t_poac.txt
