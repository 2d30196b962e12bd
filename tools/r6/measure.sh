#!/bin/bash
# Round-6 measurement session on one MI355X, every figure from the same box:
# the GPU test suite (teacher-forced flips printed), smoke(), the driver's
# bench shape three times, the default long bench line, the B=4096 bench,
# rocprofv3 kernel statistics (B=256 / B=4096 / configs[4] / exploration),
# FETCH / WRITE / SQ PMC passes, the MFMA / VALU pass of the B=4096 step,
# per-launch breakdowns, the backward-kernel micro-benchmark with stage clocks
# and the occupancy probe.  Summaries -> profiles/r06 by tools/r6/collect.sh.
mkdir -p gpurun_out/r6m
R=$PWD
O=$R/gpurun_out/r6m
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gputest_final.txt 2>&1; crash $?
tail -1 $O/gputest_final.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; crash $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_shape_$i.json 2>$O/bench_driver_shape.err; crash $?
  python3 -c "import json;d=json.loads(open('$O/bench_driver_shape_$i.json').read().strip().splitlines()[-1]);print('driver shape',d['value'],d['roofline']['frac'])"
done
timeout -k 10 500 python bench.py > $O/bench256.log 2>&1; crash $?
tail -1 $O/bench256.log | cut -c1-300
timeout -k 10 300 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline --no-extras > $O/bench4096.log 2>&1; crash $?
