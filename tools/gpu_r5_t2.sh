#!/bin/bash
# round 5: which large-batch launches take the register-direct kernel (cfg 2 / 3,
# gemm_big.hip) by default -- OAC_DEBUG_CFG prints every GEMM launch's kernel
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
OAC_DEBUG_CFG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_goac.py tests/test_gpu_ptrain.py tests/test_gpu_particle.py tests/test_gpu_ragged.py tests/test_gpu_parity.py -q -x -s -k "large or ragged or slabs or b4096 or poac_ant" $T > gpurun_out/r5_t2_cfg.log 2>&1
rc=$?; crash $rc; tail -3 gpurun_out/r5_t2_cfg.log
grep -c "^launch" gpurun_out/r5_t2_cfg.log; grep "^launch" gpurun_out/r5_t2_cfg.log | awk '{print $4}' | sort | uniq -c
grep -E "^launch [0-9]+ cfg (2|3) " gpurun_out/r5_t2_cfg.log | sort | uniq -c | sort -rn | head -20
