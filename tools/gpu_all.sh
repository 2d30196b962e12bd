#!/bin/bash
# full GPU test suite (one pytest process), then the default bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log; grep -E "FAIL|Error" gpurun_out/pytest_all.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_default.log; exit $rc
