#!/bin/bash
# round 4 A/B on one box: the wide-slab Adam pass (OAC_ADAM_WIDE) and the
# large-batch index staging (hipMemcpyAsync / copy kernel OAC_IDX_COPY=1 /
# tiles reading the host ring OAC_BIG_HOST_IDX=1), SAC B=4096 and configs[4];
# the drop-in parity tests under each staging variant first
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
for v in "OAC_IDX_COPY=0" "OAC_IDX_COPY=1" "OAC_BIG_HOST_IDX=1"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_particle.py -q -x $T > gpurun_out/r4_t6_$v.log 2>&1
  rc=$?; crash $rc; echo "$v tests rc=$rc: $(tail -1 gpurun_out/r4_t6_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in "OAC_ADAM_WIDE=0" "OAC_ADAM_WIDE=1" "OAC_IDX_COPY=1" "OAC_BIG_HOST_IDX=1"; do
    for w in "--batch 4096" "--batch 4096 --poac"; do
      env $v timeout -k 10 200 python tools/launch_times.py $w > gpurun_out/lt_t6.log 2>&1; crash $?
      echo "$v $w: $(grep -v amdgpu gpurun_out/lt_t6.log | head -1)"
      [ $i -eq 2 ] && grep -E "adam" gpurun_out/lt_t6.log | head -3
    done
  done
done
