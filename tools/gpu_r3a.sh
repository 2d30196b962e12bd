#!/bin/bash
# Round 3, first GPU pass: the GPU suite, smoke(), the driver's bench command,
# the rocprofv3 kernel statistics of the headline step and of the exploration
# call.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b256 -- python3 $R/bench.py --steps 400 --warmup 40 --no-extras --no-cpu-baseline > $R/gpurun_out/prof_b256.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_expl -- python3 $R/tools/expl_prof.py > $R/gpurun_out/prof_expl.log 2>&1
rc=$?
cd $R
tail -3 gpurun_out/gputest.log
tail -1 gpurun_out/bench_drv.log | cut -c1-600
exit $rc
