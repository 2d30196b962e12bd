#!/bin/bash
# round 6: the visible GPU's NUMA node, then the driver-shaped line pinned to
# 8 cores on each NUMA node (taskset before python; bench.py --no-pin)
O=$PWD/gpurun_out/r6/numa
mkdir -p $O
timeout -k 10 120 python3 -c "
import torch
p = torch.cuda.get_device_properties(0)
print([a for a in dir(p) if not a.startswith('_')])
for a in ('pci_bus_id', 'pci_device_id', 'pci_domain_id'):
    print(a, getattr(p, a, None))
" > $O/props.txt 2>&1; cat $O/props.txt | grep -v amdgpu.ids
for f in /sys/bus/pci/devices/*/numa_node; do d=$(dirname $f); c=$(cat $d/class 2>/dev/null); case $c in 0x038000|0x030000|0x120000) echo "$d class $c numa $(cat $f)";; esac; done > $O/pci.txt 2>&1; head -20 $O/pci.txt
for i in 1 2 3; do
  for node in 0 1; do
    cores=$( [ $node = 0 ] && echo 0-7 || echo 64-71 )
    timeout -k 10 200 taskset -c $cores python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --no-pin > $O/n${node}_$i.json 2>$O/err.txt || { echo "bench failed"; tail -5 $O/err.txt; exit 1; }
    echo "node$node $i $(python3 -c "import json;print(json.loads(open('$O/n${node}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
