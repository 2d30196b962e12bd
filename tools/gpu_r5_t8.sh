#!/bin/bash
# round 5: driver shape after moving the collection before the warm-up (3 runs),
# then the whole GPU suite on the tree without the register-direct kernel
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r5_t8_drv$i.json 2>/dev/null; rc=$?; crash $rc
  python -c "import json; d=json.loads(open('gpurun_out/r5_t8_drv$i.json').read().strip().splitlines()[-1]); print('driver shape', d['value'], d['ms_per_step'])"
done
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 > gpurun_out/r5_t8_fill.txt 2>&1; rc=$?; crash $rc; tail -7 gpurun_out/r5_t8_fill.txt | cut -c1-500
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5_t8_pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/r5_t8_pytest.txt; exit $rc
