#!/bin/bash
# Sweep GEMM tuning environments at batch 4096: large-batch GPU parity tests
# + a bench line per setting.  ENVS="A=1,B=2 A=0" (semicolon-separated per run).
set -o pipefail
mkdir -p gpurun_out
i=0
for e in $ENVS; do
  i=$((i+1))
  envs=$(echo $e | tr ';' ' ')
  env $envs timeout -k 10 300 python -u -m pytest tests/test_gpu_goac.py tests/test_gpu_parity.py \
    tests/test_gpu_particle.py tests/test_gpu_ptrain.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/env_pytest_$i.log 2>&1 || { echo "[$e] tests failed"; tail -30 gpurun_out/env_pytest_$i.log; exit 1; }
  env $envs timeout -k 10 200 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline --no-extras \
    > gpurun_out/env_bench_$i.log 2>&1 || { tail -20 gpurun_out/env_bench_$i.log; exit 1; }
  echo "[$e]: $(tail -1 gpurun_out/env_pytest_$i.log) | $(tail -1 gpurun_out/env_bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
