#!/bin/bash
# Round-6 measurement session, part B (tools/r6/measure.sh is part A): rocprofv3
# kernel statistics, PMC passes, per-launch times, micro-benchmarks.
mkdir -p gpurun_out/r6m
R=$PWD
O=$R/gpurun_out/r6m
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
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
