#!/bin/bash
# policy_head: head operands issued before the step-3 prefetch (branch-free)
mkdir -p gpurun_out
timeout -k 5 60 tools/micro/head_micro 4096 1 || exit $?
timeout -k 5 60 tools/micro/head_micro 256 4 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "sac_step or ragged or particle or goac or ptrain or dropin or eval" > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_h.log; grep -E "^FAILED|Error" gpurun_out/pytest_h.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 600 > gpurun_out/lt4096.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt4096.log | tail -16 | sed -n '1p;5p'
timeout -k 5 120 python tools/launch_times.py --batch 256 --steps 10 --rate-steps 4000 > gpurun_out/lt256.log 2>&1 || exit $?
grep -v "^launch" gpurun_out/lt256.log | tail -13 | sed -n '1p;4p'
