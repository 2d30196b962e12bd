#!/bin/bash
# Session re-entry check on one MI355X: GPU suite, smoke, the driver's bench
# shape twice, B=256 per-launch times.  Output under gpurun_out/r7.
O=$PWD/gpurun_out/r7
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.txt 2>&1; crash $?
tail -1 $O/gputests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; crash $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_ds_$i.json 2>$O/bench_ds.err; crash $?
  python3 -c "import json;d=json.loads(open('$O/bench_ds_$i.json').read().strip().splitlines()[-1]);print('driver shape',d['value'],d['roofline']['frac'])"
done
timeout -k 10 200 python tools/launch_times.py --batch 256 > $O/lt256.txt 2>&1; crash $?
cat $O/lt256.txt
