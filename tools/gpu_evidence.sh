#!/bin/bash
# per-launch breakdowns (drop-in step, hipExtLaunchKernel events) and the
# configs[4] rocprofv3 kernel statistics, for profiles/r02
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 40 --rate-steps 4000 > gpurun_out/ev_lt256.log 2>&1 &&
timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ev_lt4096.log 2>&1 &&
timeout -k 5 120 python tools/launch_times.py --poac --batch 4096 --steps 20 --rate-steps 600 > gpurun_out/ev_ltpoac.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_poac4096 -- python3 $R/tools/launch_times.py --poac --batch 4096 --steps 4 --rate-steps 200 > $R/gpurun_out/prof_poac4096.log 2>&1
rc=$?; cd $R; grep "drop-in" gpurun_out/ev_lt*.log; exit $rc
