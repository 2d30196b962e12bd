#!/bin/bash
# A/B of step-structure switches at batch 256 on one box, interleaved twice.
# CASES="name:ENV=1;ENV2=0 ..."   -> one bench line per case and repetition
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for c in $CASES; do
    name=${c%%:*}; envs=$(echo ${c#*:} | tr ';' ' ')
    env $envs timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --steps 1280 --warmup 64 ${BENCH_ARGS} \
      > gpurun_out/ab_${name}_$rep.log 2>&1 || { tail -20 gpurun_out/ab_${name}_$rep.log; exit 1; }
    echo "$name rep$rep $(tail -1 gpurun_out/ab_${name}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
