#!/bin/bash
# round 5 final: the full GPU suite and smoke on the final tree, then the
# measurement session (tools/measure_r5.sh) whose files go to profiles/r05
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pytest_all.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1; rc=$?; crash $rc; tail -2 gpurun_out/r5_smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/measure_r5.sh
