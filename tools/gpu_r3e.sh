#!/bin/bash
# exploration stage clocks; backward default (cfg 12) parity + B=4096 launch times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/expl_micro 300 > gpurun_out/expl_micro.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_altkernels.py tests/test_gpu_ragged.py tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_goac.py tests/test_gpu_ptrain.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/bwd_tests.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 &&
timeout -k 10 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ltpoac.log 2>&1
rc=$?
cat gpurun_out/expl_micro.log; tail -2 gpurun_out/bwd_tests.log; cat gpurun_out/lt4096.log gpurun_out/ltpoac.log | grep -v amdgpu.ids
exit $rc
