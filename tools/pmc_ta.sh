#!/bin/bash
# round 4: the texture-address / L1 counters of the B=256 step (one pass each,
# kernel trace only): is the small kernel's fragment-shaped operand fetch
# (64 lanes = 64 cache lines per 16-B load) what its launches wait on?
# usage: tools/pmc_ta.sh <tag> [bench args...] -> gpurun_out/pmc_<tag>_ta*, counter list
TAG=$1; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/rocprof_counters_list.txt 2>&1 || true
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$1 \
    -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 --steps-per-launch 1 "${@:3}" \
    > $R/gpurun_out/pmc_${TAG}_$1.log 2>&1
}
run ta "TA_BUSY_avr TA_BUSY_max SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" "$@"
run tcp "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" "$@"
exit 0
