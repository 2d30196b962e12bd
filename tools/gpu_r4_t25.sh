#!/bin/bash
# round 4 A/B at B=256: critic layer-1 Adam previewed into the shadow (p only), the full update as side blocks of the layer-0 launch
# (new) or before it (base: in-order vmcnt makes the first MFMA wait for them)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_teacher.py tests/test_gpu_ring.py -q -x $T > gpurun_out/r4_t25_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r4_t25_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base new; do
    L=oac-explore_amd/oac_amd/liboac_amd.so; [ $v = base ] && L=oac-explore_amd/oac_amd/liboac_amd_base.so
    OAC_LIB=$PWD/$L timeout -k 10 200 python tools/launch_times.py > gpurun_out/r4_t25_lt_$v.log 2>&1; crash $?
    echo "$v $(grep drop-in gpurun_out/r4_t25_lt_$v.log)"
  done
done
grep 'launch ' gpurun_out/r4_t25_lt_new.log | tr -s ' ' | tr '\n' '|'; echo
