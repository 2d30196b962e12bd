#!/bin/bash
# exploration A/B, the full GPU suite, then per-launch times (with the
# launch configurations) at B=4096 and configs[4]
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/expl_ab.log
for i in 1 2; do
  timeout -k 10 60 tools/micro/expl_micro 400 1 1 | head -1 >> gpurun_out/expl_ab.log &&
  timeout -k 10 60 tools/micro/expl_micro 400 1 0 | head -1 >> gpurun_out/expl_ab.log || exit 1
done
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/expl_micro.log 2>&1 || exit 1
cat gpurun_out/expl_ab.log gpurun_out/expl_micro.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
OAC_DEBUG_CFG=1 timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 2 --rate-steps 10 > gpurun_out/cfg_b4096.log 2>&1 &&
timeout -k 10 200 python tools/launch_times.py --batch 4096 > gpurun_out/lt_b4096.log 2>&1 &&
timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/lt_poac.log 2>&1 &&
timeout -k 10 120 python tools/expl_prof.py > gpurun_out/expl_wall.log 2>&1
rc=$?
grep "launch .* cfg" gpurun_out/cfg_b4096.log | head -14
tail -n 16 gpurun_out/lt_b4096.log; tail -n 20 gpurun_out/lt_poac.log; tail -1 gpurun_out/expl_wall.log
exit $rc
