#!/bin/bash
# round 6: policy_head_kernel stage clocks at B=4096 (one column chunk, the
# large-batch form) and B=256
O=$PWD/gpurun_out/r6/head
mkdir -p $O
timeout -k 5 60 tools/micro/head_micro 4096 1 > $O/head_4096.txt 2>&1 || exit $?
timeout -k 5 60 tools/micro/head_micro 4096 2 > $O/head_4096_cc2.txt 2>&1 || exit $?
timeout -k 5 60 tools/micro/head_micro 256 4 > $O/head_256.txt 2>&1 || exit $?
cat $O/head_4096.txt $O/head_4096_cc2.txt $O/head_256.txt | grep -v amdgpu.ids
