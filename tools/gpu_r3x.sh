#!/bin/bash
# timing experiment: the B=4096 critic layer-1 backward launch without its dW-last tiles (1152 -> 1024 workgroups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/launch_times.py --batch 4096 > gpurun_out/lt_x0.txt 2>&1 &&
OAC_EXP_NO_DWLAST=1 timeout -k 10 300 python tools/launch_times.py --batch 4096 > gpurun_out/lt_x1.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/lt_x0.txt; grep -v amdgpu.ids gpurun_out/lt_x1.txt
exit $rc
