#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_dropin.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dpov.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dpov.log; grep -E "^FAILED|Error" gpurun_out/pytest_dpov.log | head -5; [ $rc -eq 0 ] || exit $rc
for ov in 1 0; do
  OAC_DP_OVERLAP=$ov OAC_BENCH_FORCE_DP=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --no-cpu-baseline --no-extras --steps 400 --warmup 40 > gpurun_out/dpov_$ov.log 2>&1 || exit 1
  echo "overlap=$ov $(tail -1 gpurun_out/dpov_$ov.log | cut -c1-200)"
done
