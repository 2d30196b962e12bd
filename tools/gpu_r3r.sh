#!/bin/bash
# small-batch direct gather: one index read per workgroup / side row -- tests + B=256 launch times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_ring.py -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3r_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3r_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python tools/launch_times.py --batch 256 2>&1 | grep -v amdgpu.ids | head -14 || exit 1
done
