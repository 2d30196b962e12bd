#!/bin/bash
# round 4 A/B at B=256: the fused Adam's step constants (a dependent read of
# the step state) computed before the small kernel's k loop (new) or in its
# epilogue (base); gemm_micro stage clocks of the fused-Adam dW batch
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 120 tools/micro/gemm_micro > gpurun_out/r4_gemm_micro3.log 2>&1 || exit 1
grep -A1 "Adam" gpurun_out/r4_gemm_micro3.log | grep -A1 "nw  0"
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_teacher.py -q -x $T > gpurun_out/r4_t19_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r4_t19_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base new; do
    L=oac-explore_amd/oac_amd/liboac_amd.so; [ $v = base ] && L=oac-explore_amd/oac_amd/liboac_amd_base.so
    OAC_LIB=$PWD/$L timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t19_lt_$v.log 2>&1; crash $?
    echo "$v $(grep drop-in gpurun_out/r4_t19_lt_$v.log)"
  done
done
grep 'launch ' gpurun_out/r4_t19_lt_new.log | tr -s ' ' | tr '\n' '|'; echo
