#!/bin/bash
# policy_head at large batch: micro (cc 1 / 2), SAC parity at every batch, per-launch times at B=4096
mkdir -p gpurun_out
for cc in 1 2; do timeout -k 5 60 tools/micro/head_micro 4096 $cc || exit $?; done
timeout -k 5 60 tools/micro/head_micro 256 4 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ragged.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "sac_step or ragged" > gpurun_out/pytest_head.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 300 > gpurun_out/lt4096.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096.log | tail -18
OAC_HEAD_CC=2 timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 20 --rate-steps 300 > gpurun_out/lt4096b.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096b.log | head -2
