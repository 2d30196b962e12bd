#!/bin/bash
# round 5, final tree: the bench's N > 1 path rehearsed on one GPU (two ranks,
# gloo transport on the same device) -- the code the driver's scaling runs take
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
OAC_BENCH_BACKEND=gloo OAC_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r5_t34_n2.log 2>&1; rc=$?; crash $rc
tail -1 gpurun_out/r5_t34_n2.log | cut -c1-400; exit $rc
