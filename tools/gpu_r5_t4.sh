#!/bin/bash
# round 5: the driver's command shape (3 runs), the window decomposition with
# pre-created events, and the large-batch kernel-selection census
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r5_t4_drv$i.json 2>/dev/null; rc=$?; crash $rc
  python -c "import json; d=json.loads(open('gpurun_out/r5_t4_drv$i.json').read().strip().splitlines()[-1]); print('driver shape', d['value'], d['ms_per_step'])"
done
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 > gpurun_out/r5_t4_fill.txt 2>&1; rc=$?; crash $rc; tail -7 gpurun_out/r5_t4_fill.txt | cut -c1-700
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 --events 0 > gpurun_out/r5_t4_fill0.txt 2>&1; rc=$?; crash $rc; tail -3 gpurun_out/r5_t4_fill0.txt | cut -c1-400
bash tools/gpu_r5_t2.sh
