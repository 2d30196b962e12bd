#!/bin/bash
# quick loop: SAC parity + drop-in tests, then the B=256 headline (no extras)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_ring.py tests/test_gpu_ragged.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python bench.py --steps 3000 --warmup 300 --no-extras --no-cpu-baseline > gpurun_out/bq.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['launches_per_step'], d['kernels']['row'])"
done
