#!/bin/bash
# exploration A/B + tests, then the backward pipeline's per-stage clocks
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r3n.sh && \
timeout -k 10 120 tools/micro/bwd_clock_micro 12 10 > gpurun_out/bwd_clock.log 2>&1
rc=$?
cat gpurun_out/bwd_clock.log
exit $rc
