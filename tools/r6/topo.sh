#!/bin/bash
# round 6: the GPU box's CPU / GPU topology (KFD nodes, NUMA nodes, visible devices)
O=$PWD/gpurun_out/r6/topo
mkdir -p $O
{
  env | grep -E "VISIBLE|OMP_NUM|GPU_MAX" ; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
  for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
  for p in /sys/class/kfd/kfd/topology/nodes/*; do
    echo "== $p"; grep -E "cpu_cores_count|simd_count|location_id|domain|drm_render_minor|gpu_id" $p/properties | tr '\n' ' '; echo
    for l in $p/io_links/*; do [ -f $l/properties ] && grep -E "node_from|node_to|type|weight" $l/properties | tr '\n' ' ' && echo; done
  done
  ls -l /dev/dri/ 2>/dev/null | head -20
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
} > $O/topo.txt 2>&1
cat $O/topo.txt | head -120
