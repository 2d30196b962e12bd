#!/bin/bash
# round-4 baseline on a fresh box: the GPU suite, then the default bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_base.log 2>&1
rc=$?; tail -3 gpurun_out/r4_pytest_base.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r4_bench_base.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench_base.log | cut -c1-400
