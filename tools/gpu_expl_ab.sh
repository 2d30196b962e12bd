#!/bin/bash
# exploration latency over workgroup size x group cap (tools/expl_latency.py)
mkdir -p gpurun_out
for th in 256 512 1024; do for g in 8 16 32; do
  echo "threads=$th group=$g"
  OAC_EXPL_THREADS=$th OAC_EXPL_GROUP=$g timeout -k 10 120 python tools/expl_latency.py 2>&1 | grep full_call || exit 1
done; done
