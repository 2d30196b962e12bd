#!/bin/bash
# round 6: the MFMA / VALU / wait counters of the B=4096 step with the default
# backward kernel (cfg 12), the software-pipelined loop (cfg 17) and the
# 16-deep 4-stage ring (cfg 15), one pass each (kernel trace only)
R=$PWD
O=$R/gpurun_out/r6/pmcvar
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32"
for cfg in 12 17 15; do
  OAC_TUNE=bwdp_cfg=$cfg timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/cfg$cfg \
    -- python3 $R/tools/launch_times.py --batch 4096 --steps 8 --rate-steps 100 > $O/cfg$cfg.log 2>&1
  echo "cfg $cfg rc=$?"
done
