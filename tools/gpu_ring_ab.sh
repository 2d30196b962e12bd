#!/bin/bash
# ring path: steps per graph launch
mkdir -p gpurun_out
for n in 1 4 8 16 64; do
  timeout -k 10 200 python bench.py --mode ring --steps 1280 --warmup 64 --steps-per-launch $n --no-cpu-baseline --no-extras > gpurun_out/ring_$n.log 2>&1 || exit $?
  echo "n=$n: $(tail -1 gpurun_out/ring_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["loop"])')"
done
