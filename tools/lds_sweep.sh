#!/bin/bash
# Sweep the LDS GEMM tile variants (OAC_LDS_TILE) at batch 4096: large-batch
# GPU parity tests + a bench line per variant.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  OAC_LDS_TILE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_goac.py tests/test_gpu_parity.py \
    tests/test_gpu_particle.py tests/test_gpu_ptrain.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/lds_pytest_$v.log 2>&1 || { echo "variant $v tests failed"; tail -20 gpurun_out/lds_pytest_$v.log; exit 1; }
  OAC_LDS_TILE=$v timeout -k 10 200 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline --no-extras \
    > gpurun_out/lds_bench_$v.log 2>&1 || exit 1
  echo "variant $v: $(tail -1 gpurun_out/lds_pytest_$v.log) | $(tail -1 gpurun_out/lds_bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
