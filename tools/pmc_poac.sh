#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per pass, kernel trace
# only) over the configs[4] P-OAC workload (tools/launch_times.py --poac)
#   -> gpurun_out/pmc_poac4096_{fetch,write}
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
for k in fetch:FETCH_SIZE write:WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc ${k#*:} --kernel-trace --output-format csv -d $R/gpurun_out/pmc_poac4096_${k%%:*} \
    -- python3 $R/tools/launch_times.py --poac --batch 4096 --steps 4 --rate-steps 16 \
    > $R/gpurun_out/pmc_poac4096_${k%%:*}.log 2>&1
done
