#!/bin/bash
# the driver's bench command shape (--steps 20 --warmup 5), three runs
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_drv_$i.log 2>&1; crash $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r4_drv_$i.log').read().strip().splitlines()[-1]);print('run $i', d['value'], d['ms_per_step'])"
done
