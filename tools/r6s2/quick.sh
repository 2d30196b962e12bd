#!/bin/bash
# Focused GPU tests of a change (pytest -k expression $1), then B=256
# per-launch times and the driver's bench shape twice.  Output: gpurun_out/r7.
O=$PWD/gpurun_out/r7
mkdir -p $O
TAG=${TAG:-q}
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -k "$1" > $O/tests_$TAG.txt 2>&1; rc=$?
tail -3 $O/tests_$TAG.txt; crash $rc
timeout -k 10 200 python tools/launch_times.py --batch 256 > $O/lt256_$TAG.txt 2>&1; crash $?
cat $O/lt256_$TAG.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_${TAG}_$i.json 2>$O/bench_$TAG.err; crash $?
  python3 -c "import json;d=json.loads(open('$O/bench_${TAG}_$i.json').read().strip().splitlines()[-1]);print('driver shape',d['value'],d['roofline']['frac'])"
done
