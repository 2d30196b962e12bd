#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel trace only, never
# combined with other trace domains) over a short bench run:
#   pass 1 FETCH_SIZE, pass 2 WRITE_SIZE, pass 3 SQ wave-state counters.
# usage: tools/pmc.sh <tag> [bench args...]   -> gpurun_out/pmc_<tag>_{fetch,write,sq}
set -e
TAG=$1; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$1 \
    -- python3 $R/bench.py --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 --steps-per-launch 1 "${@:3}" \
    > $R/gpurun_out/pmc_${TAG}_$1.log 2>&1
}
run fetch FETCH_SIZE "$@"
run write WRITE_SIZE "$@"
run sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32" "$@"
