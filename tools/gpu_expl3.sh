#!/bin/bash
# exploration kernel: parity tests, then host wall per call and rocprofv3 stats
set -o pipefail
mkdir -p gpurun_out
R=$PWD
rm -rf gpurun_out/prof_expl
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_parity.py tests/test_rollout.py -x -q -m gpu --timeout 120 --timeout-method thread -k "expl or rollout or eval or predict" > gpurun_out/expl_tests.log 2>&1 &&
timeout -k 10 120 python tools/expl_prof.py > gpurun_out/expl_wall.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_expl -- python3 $R/tools/expl_prof.py > $R/gpurun_out/prof_expl.log 2>&1
rc=$?
cd $R
tail -3 gpurun_out/expl_tests.log; cat gpurun_out/expl_wall.log | tail -2
exit $rc
