#!/bin/bash
# round 6, after the backward-kernel variants and the last-arrival Adam: the
# GPU suite, smoke(), the driver's bench shape, and a same-box A/B of this
# build (cur2) against the build before them (sm16) at B=256 / 4096 / configs[4]
O=$PWD/gpurun_out/r6v
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gputest_final.txt 2>&1; crash $?
tail -1 $O/gputest_final.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; crash $?
tail -2 $O/smoke.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_shape_$i.json 2>$O/bench_driver_shape.err; crash $?
  python3 -c "import json;d=json.loads(open('$O/bench_driver_shape_$i.json').read().strip().splitlines()[-1]);print('driver shape',d['value'],d['roofline']['frac'])"
done
TAG=val VARIANTS="sm16 cur2" LEGS="b256 b4096 poac" ROUNDS=2 bash tools/r6/ab_libs.sh
