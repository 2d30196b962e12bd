#!/bin/bash
# round 4: new tests, exploration parity + micro, the staged small kernel's parity subset and A/B, TA counters, full suite
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r4_new_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|worst|Error" gpurun_out/r4_new_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "expl or philox" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_expl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_expl_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/r4_expl_micro.log 2>&1 || exit 1
cat gpurun_out/r4_expl_micro.log | head -20
OAC_SMALL_STAGE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ring.py tests/test_gpu_ragged.py tests/test_gpu_teacher.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_stage_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_stage_tests.log; [ $rc -eq 0 ] || exit $rc
OAC_PBWD_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ring.py tests/test_gpu_teacher.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pbwd_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_pbwd_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_stage.sh || exit 1
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro.log 2>&1 || exit 1
OAC_SMALL_STAGE=1 timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro_stage.log 2>&1 || exit 1
bash tools/pmc_ta.sh b256
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/r4_pytest_all.log; [ $rc -eq 0 ] || exit $rc
