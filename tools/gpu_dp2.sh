#!/bin/bash
# data-parallel alpha exchange over the head launch's logp partials: DP tests + 2-rank rehearsal
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dp or checkpoint or sac_step" > gpurun_out/pytest_dp.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dp.log; grep -E "^FAILED|Error" gpurun_out/pytest_dp.log | head; [ $rc -eq 0 ] || exit $rc
OAC_BENCH_SAME_DEVICE=1 OAC_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 8 --no-cpu-baseline --no-extras > gpurun_out/bench_g2.log 2>&1 || { tail -20 gpurun_out/bench_g2.log; exit 1; }
tail -1 gpurun_out/bench_g2.log | cut -c1-150
