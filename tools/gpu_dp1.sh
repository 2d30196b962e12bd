#!/bin/bash
# data-parallel step structure at one rank (RCCL, graph-captured): alpha-exchange overlap on / off
mkdir -p gpurun_out
for b in 256 4096; do
for v in 1 0; do
  OAC_BENCH_FORCE_DP=1 OAC_DP_OVERLAP=$v timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
     bench.py --gpus 1 --batch $b --steps 200 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/dp1_${b}_$v.log 2>&1; rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { grep -v "^{" gpurun_out/dp1_${b}_$v.log | tail -5; exit $rc; }
  echo "B=$b overlap=$v: $(tail -1 gpurun_out/dp1_${b}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("mode"))')"
done
done
