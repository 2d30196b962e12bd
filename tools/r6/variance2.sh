#!/bin/bash
# round 6: the driver-shaped bench line with bench.py's own host pinning
# (default) against --no-pin, interleaved on one box; then one default run
# (the CPU baseline's all-cores leg must still see every core)
O=$PWD/gpurun_out/r6/var2
mkdir -p $O
for i in 1 2 3 4 5 6; do
  for mode in pin nopin; do
    F=""; [ $mode = nopin ] && F="--no-pin"
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras $F > $O/${mode}_$i.json 2>$O/err.txt || { echo "bench failed"; tail -5 $O/err.txt; exit 1; }
    echo "$mode $i $(python3 -c "import json;print(json.loads(open('$O/${mode}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
timeout -k 10 500 python bench.py > $O/default.json 2>$O/err_default.txt || { echo "default bench failed"; tail -5 $O/err_default.txt; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/default.json').read().strip().splitlines()[-1])
print('default', d['value'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('all_cores',{}).get('value'), d['cpu_baseline'].get('all_cores',{}).get('cores'), 'b4096', d['b4096']['steps_per_s'], 'poac', d['poac_ant_b4096']['steps_per_s'], 'expl', d['exploration']['us_per_call_1obs'])"
