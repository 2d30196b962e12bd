#!/bin/bash
# Round-6 second-session measurement on one MI355X (final tree): the GPU test
# suite, smoke(), the driver's bench shape three times, the default bench line
# (CPU baselines and extra legs), rocprofv3 kernel statistics and the
# FETCH / WRITE PMC passes of the B=256 step, per-launch times.
# Summaries -> profiles/r06 by tools/r6s2/collect.sh.
mkdir -p gpurun_out/r6f
R=$PWD
O=$R/gpurun_out/r6f
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gputest_final.txt 2>&1; crash $?
tail -1 $O/gputest_final.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; crash $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_shape_$i.json 2>$O/bench_driver_shape.err; crash $?
  python3 -c "import json;d=json.loads(open('$O/bench_driver_shape_$i.json').read().strip().splitlines()[-1]);print('driver shape',d['value'],d['roofline']['frac'])"
done
timeout -k 10 200 python tools/launch_times.py --batch 256 > $O/lt_b256.log 2>&1; crash $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b256 -- \
  python3 $R/bench.py --steps 160 --warmup 32 --no-cpu-baseline --no-extras --timing-steps 8 > $O/prof_b256.log 2>&1; crash $?
pmc() {  # tag, counters
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/pmc_$1 \
    -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 --steps-per-launch 1 \
    > $O/pmc_$1.log 2>&1
}
pmc b256_fetch FETCH_SIZE; crash $?
pmc b256_write WRITE_SIZE; crash $?
pmc b256_sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32"; crash $?
cd $R
timeout -k 10 600 python bench.py > $O/bench256.log 2>&1; crash $?
tail -1 $O/bench256.log | cut -c1-400
