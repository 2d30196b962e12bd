#!/bin/bash
# policy head kernel at B=4096 (one column chunk, as the step runs it): launch time and stage clocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/head_micro 4096 1 > gpurun_out/head_micro.txt 2>&1 && timeout -k 10 60 tools/micro/head_micro 4096 2 >> gpurun_out/head_micro.txt 2>&1
rc=$?
cat gpurun_out/head_micro.txt
exit $rc
