#!/bin/bash
# round 4: the new teacher-forced / mid-state / forced-overlap DP tests first,
# then the whole GPU suite and the default bench line
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r4_new_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|worst|Error" gpurun_out/r4_new_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/r4_pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r4_bench_base.log 2>&1 || exit 1
tail -1 gpurun_out/r4_bench_base.log | cut -c1-600
