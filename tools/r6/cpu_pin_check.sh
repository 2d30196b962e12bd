#!/bin/bash
# round 6: the CPU baseline's all-cores leg with bench.py pinning (then
# unpinning) against --no-pin, same box, twice each
O=$PWD/gpurun_out/r6/cpupin2
mkdir -p $O
for i in 1 2; do
  for F in ""; do
    tag=${F:-pin}
    timeout -k 10 500 python bench.py --no-extras $F > $O/b_${tag}_$i.json 2>$O/err.txt || { echo "bench failed"; tail -5 $O/err.txt; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${tag}_$i.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']
print('$tag $i', d['value'], 'cpu1', c['value'], 'all', c['all_cores']['value'], c['all_cores']['runs'])"
  done
done
