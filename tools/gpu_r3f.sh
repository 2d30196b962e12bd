#!/bin/bash
# exploration: da in S4 parts (stage clocks, tests, wall); tile sweep of the
# large-batch launches (SAC B=4096 and configs[4]) through the A/B switches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/expl_micro 300 > gpurun_out/expl_micro.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parity.py tests/test_rollout.py -x -q -m gpu --timeout 120 --timeout-method thread -k "expl or rollout or eval or predict" > gpurun_out/expl_tests.log 2>&1 &&
timeout -k 10 120 python tools/expl_prof.py > gpurun_out/expl_wall.log 2>&1 || exit 1
cat gpurun_out/expl_micro.log; tail -2 gpurun_out/expl_tests.log; tail -1 gpurun_out/expl_wall.log
: > gpurun_out/sweep.log
for v in "" "OAC_FWD2_TILE=64,64" "OAC_FWD2_TILE=128,128" "OAC_FWD2_TILE=64,64 OAC_FWD2_NB=2" "OAC_BWDP_CFG=9"; do
  echo "== $v" >> gpurun_out/sweep.log
  env $v timeout -k 10 90 python tools/launch_times.py --poac --batch 4096 --steps 4 --rate-steps 600 2>&1 | grep drop-in >> gpurun_out/sweep.log || exit 1
  env $v timeout -k 10 90 python tools/launch_times.py --batch 4096 --steps 4 --rate-steps 600 2>&1 | grep drop-in >> gpurun_out/sweep.log || exit 1
done
cat gpurun_out/sweep.log
