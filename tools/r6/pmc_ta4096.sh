#!/bin/bash
# round 6: vector-memory (TA / TD / TCP) counters of the B=4096 SAC step's
# kernels, one pass each, kernel trace only: is the backward GEMM's operand
# intake (~12 B/cycle/CU) the address / data path's
# limit?  -> gpurun_out/r6/pmcta/*, counter list
R=$PWD
O=$R/gpurun_out/r6/pmcta
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/$1 \
    -- python3 $R/bench.py --batch 4096 --steps 32 --warmup 16 --no-cpu-baseline --no-extras --timing-steps 4 \
    > $O/$1.log 2>&1
  echo "pass $1 rc=$?"
}
run ta "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"
run td "TD_BUSY_avr TD_BUSY_max GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"
run tcp "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"
exit 0
