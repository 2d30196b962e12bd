#!/bin/bash
# XCD mapping of an exploration-shaped launch, and flag round-trip latency same-XCD / cross-XCD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/micro/xcd_probe 256 > gpurun_out/xcd_probe.txt 2>&1 && timeout -k 10 60 tools/micro/xcd_probe 64 >> gpurun_out/xcd_probe.txt 2>&1 && timeout -k 10 60 tools/micro/xcd_probe 256 2000 >> gpurun_out/xcd_probe.txt 2>&1
rc=$?
cat gpurun_out/xcd_probe.txt
exit $rc
