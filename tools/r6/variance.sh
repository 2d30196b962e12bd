#!/bin/bash
# round 6: spread of the driver-shaped bench line (20 steps after 5) over
# repeated runs on one box, as is and with the process on 8 fixed cores
O=$PWD/gpurun_out/r6/var
mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpuset.cpus.effective > $O/cpus.txt 2>/dev/null || true
for i in 1 2 3 4 5 6; do
  for mode in free pin; do
    if [ $mode = pin ]; then P="taskset -c $(python3 -c "import os;c=sorted(os.sched_getaffinity(0));print(','.join(map(str,c[:8])))")"; else P=""; fi
    timeout -k 10 200 $P python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/${mode}_$i.json 2>$O/err.txt || { echo "bench failed"; tail -5 $O/err.txt; exit 1; }
    echo "$mode $i $(python3 -c "import json;print(json.loads(open('$O/${mode}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
