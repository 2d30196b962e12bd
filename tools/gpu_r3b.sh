#!/bin/bash
# Round 3: the driver's bench command and the rocprofv3 kernel statistics of
# the headline step and of the exploration call.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b256 -- python3 $R/bench.py --steps 400 --warmup 40 --no-extras --no-cpu-baseline > $R/gpurun_out/prof_b256.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_expl -- python3 $R/tools/expl_prof.py > $R/gpurun_out/prof_expl.log 2>&1
rc=$?
cd $R
tail -1 gpurun_out/bench_drv.log | cut -c1-600
exit $rc
