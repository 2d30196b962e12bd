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
cd /tmp && export TMPDIR=/tmp
prof() {  # tag, command...
  local t=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -- "$@" > $O/prof_$t.log 2>&1
}
prof b256 python3 $R/bench.py --steps 160 --warmup 32 --no-cpu-baseline --no-extras --timing-steps 8; crash $?
prof b4096 python3 $R/bench.py --batch 4096 --steps 48 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 8; crash $?
prof poac4096 python3 $R/tools/launch_times.py --poac --batch 4096 --steps 8 --rate-steps 200; crash $?
prof expl python3 $R/tools/expl_prof.py; crash $?
pmc() {  # tag, counters, bench args...
  local t=$1 c=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$t \
    -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 --steps-per-launch 1 "$@" \
    > $O/pmc_$t.log 2>&1
}
for b in 256 4096; do
  pmc b${b}_fetch FETCH_SIZE --batch $b; crash $?
  pmc b${b}_write WRITE_SIZE --batch $b; crash $?
  pmc b${b}_sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32" --batch $b; crash $?
done
(cd $R && bash tools/pmc_poac.sh); crash $?
pmc b4096_mfma "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32" --batch 4096; crash $?
cd $R
timeout -k 10 200 python tools/launch_times.py --batch 256 > $O/lt_b256.log 2>&1; crash $?
timeout -k 10 200 python tools/launch_times.py --batch 4096 > $O/lt_b4096.log 2>&1; crash $?
timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > $O/lt_poac.log 2>&1; crash $?
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > $O/expl_micro.log 2>&1; crash $?
timeout -k 10 60 tools/micro/bwd_micro 12 1 > $O/bwd_micro.log 2>&1; crash $?
timeout -k 10 60 tools/micro/bwd_clock_micro 12 1 > $O/bwd_clock.log 2>&1; crash $?
tail -1 $O/bench256.log | cut -c1-300
