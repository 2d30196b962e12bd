#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/expl_micro 300 > gpurun_out/expl_micro.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parity.py tests/test_rollout.py -x -q -m gpu --timeout 120 --timeout-method thread -k "expl or rollout or eval or predict" > gpurun_out/expl_tests.log 2>&1 &&
timeout -k 10 120 python tools/expl_prof.py > gpurun_out/expl_wall.log 2>&1
rc=$?
cat gpurun_out/expl_micro.log; tail -2 gpurun_out/expl_tests.log; tail -1 gpurun_out/expl_wall.log
exit $rc
