#!/bin/bash
# exploration: the twin-critic kernel (one polled hand-off + one arrival)
# against the four-hand-off split kernel, then the exploration tests and the
# host wall through the Python call
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/expl_ab.log
for i in 1 2; do
  timeout -k 10 60 tools/micro/expl_micro 400 1 1 | head -1 >> gpurun_out/expl_ab.log &&
  timeout -k 10 60 tools/micro/expl_micro 400 1 0 | head -1 >> gpurun_out/expl_ab.log || exit 1
done
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/expl_micro.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parity.py tests/test_rollout.py tests/test_gpu_dropin.py -x -q -m gpu --timeout 120 --timeout-method thread -k "expl or rollout or eval or predict" > gpurun_out/expl_tests.log 2>&1 &&
timeout -k 10 120 python tools/expl_prof.py > gpurun_out/expl_wall.log 2>&1
rc=$?
cat gpurun_out/expl_ab.log gpurun_out/expl_micro.log; tail -3 gpurun_out/expl_tests.log; tail -2 gpurun_out/expl_wall.log
exit $rc
