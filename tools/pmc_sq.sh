#!/bin/bash
# one SQ PMC pass (kernel trace only) over a short bench run: tools/pmc_sq.sh <tag> [bench args]
set -e
TAG=$1; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_sq \
  -- python3 $R/bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-extras --timing-steps 2 "$@" > $R/gpurun_out/pmc_${TAG}_sq.log 2>&1
