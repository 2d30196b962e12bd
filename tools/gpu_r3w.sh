#!/bin/bash
# head kernel A/B: micro, per-launch times at B=4096, parity tests of the plans that launch it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/head_micro 4096 1 > gpurun_out/head_micro_w.txt 2>&1 &&
timeout -k 10 300 python tools/launch_times.py --batch 4096 > gpurun_out/lt_w_b4096.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_dropin.py tests/test_gpu_ragged.py > gpurun_out/w_tests.log 2>&1
rc=$?
cat gpurun_out/head_micro_w.txt; grep -v amdgpu.ids gpurun_out/lt_w_b4096.txt; tail -3 gpurun_out/w_tests.log
exit $rc
