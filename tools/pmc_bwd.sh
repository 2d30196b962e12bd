#!/bin/bash
# SQ / TA / TCC counter passes over the B=4096 launch-time run (one pass each)
R=$PWD
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmcb_$tag \
    -- python3 $R/tools/launch_times.py --batch 4096 --rate-steps 20 --steps 4 > $R/gpurun_out/pmcb_$tag.log 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD || exit 1
run sq2 SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum || exit 1
echo done
