#!/bin/bash
# round 6: the driver-shaped line pinned (taskset, bench.py --no-pin) to 2 / 4 / 8 / 16 cores
O=$PWD/gpurun_out/r6/pinsize
mkdir -p $O
for i in 1 2 3; do
  for c in 0-1 0-3 0-7 0-15; do
    timeout -k 10 200 taskset -c $c python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --no-pin > $O/c${c}_$i.json 2>$O/err.txt || { echo "bench failed"; tail -5 $O/err.txt; exit 1; }
    echo "cores $c $i $(python3 -c "import json;print(json.loads(open('$O/c${c}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
