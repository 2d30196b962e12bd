#!/bin/bash
# round 4: the full GPU suite on the final tree, smoke(), then the dataflow micro
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_all.log 2>&1
rc=$?; crash $rc; tail -4 gpurun_out/r4_pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1; rc=$?; crash $rc; tail -2 gpurun_out/r4_smoke.log
timeout -k 10 120 tools/micro/dataflow_micro > gpurun_out/r4_dataflow_micro3.log 2>&1; crash $?
cat gpurun_out/r4_dataflow_micro3.log
