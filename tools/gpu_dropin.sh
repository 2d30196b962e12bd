#!/bin/bash
# drop-in path: GPU tests, default bench, 2-rank rehearsal (gloo, one GPU)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dropin.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dropin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -c 4000 gpurun_out/bench_default.log; [ $rc -eq 0 ] || exit $rc
OAC_BENCH_SAME_DEVICE=1 OAC_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 8 --no-cpu-baseline > gpurun_out/bench_gpus2.log 2>&1
rc=$?; tail -c 1500 gpurun_out/bench_gpus2.log; exit $rc
