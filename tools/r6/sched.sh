#!/bin/bash
# round 6: the driver-shaped bench line under each HIP device schedule flag,
# interleaved on one box
O=$PWD/gpurun_out/r6/sched
mkdir -p $O
for i in 1 2 3 4; do
  for m in auto spin yield block; do
    timeout -k 10 200 python tools/r6/sched_bench.py $m --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/${m}_$i.json 2>$O/err.txt || { echo "bench failed ($m)"; tail -5 $O/err.txt; exit 1; }
    echo "$m $i $(python3 -c "import json;print(json.loads(open('$O/${m}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
