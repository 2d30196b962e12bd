#!/bin/bash
# round 6: the large-batch backward GEMM (gemm_bwdp.hip) at the B=4096 SAC
# step's backward launches -- per-launch time (tools/micro/bwd_micro), stage
# clocks, one SQ PMC pass; TAG names the output files
TAG=${TAG:-base}
CFG=${CFG:-12}
R=$PWD
O=$R/gpurun_out/r6
mkdir -p $O
crash() { case $1 in 0) ;; *) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 5 60 tools/micro/bwd_micro $CFG 1 > $O/bwd_${TAG}.txt 2>&1; crash $?
cat $O/bwd_${TAG}.txt
timeout -k 5 60 tools/micro/bwd_clock_micro $CFG 1 > $O/bwd_clock_${TAG}.txt 2>&1; crash $?
grep clocks $O/bwd_clock_${TAG}.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 \
  --kernel-trace --output-format csv -d $O/pmc_bwd_${TAG} -- $R/tools/micro/bwd_micro $CFG 1 > $O/pmc_bwd_${TAG}.log 2>&1; crash $?
cd $R
python3 tools/r6/pmc_kernels.py $O/pmc_bwd_${TAG} bwdp > $O/pmc_bwd_${TAG}.txt; cat $O/pmc_bwd_${TAG}.txt
