#!/bin/bash
# Focused GPU tests (pytest -k $1), then B=4096 / configs[4] per-launch times and
# the B=4096 bench leg.  Output: gpurun_out/r7.
O=$PWD/gpurun_out/r7
mkdir -p $O
TAG=${TAG:-b}
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -k "$1" > $O/tests_$TAG.txt 2>&1; rc=$?
tail -3 $O/tests_$TAG.txt; crash $rc
timeout -k 10 200 python tools/launch_times.py --batch 4096 > $O/lt4096_$TAG.txt 2>&1; crash $?
cat $O/lt4096_$TAG.txt
timeout -k 10 300 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline --no-extras > $O/bench4096_$TAG.json 2>$O/bench4096_$TAG.err; crash $?
python3 -c "import json;d=json.loads(open('$O/bench4096_$TAG.json').read().strip().splitlines()[-1]);print('b4096',d['value'],d['roofline']['frac'])"
