#!/bin/bash
# round 4 A/B: the LDS-DMA kernels' bank swizzle kc_swz(r) = (r >> 1) & 7
# (base: r & 7, 2-way conflicts on every ds_read_b128 fragment read)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_altkernels.py tests/test_gpu_ragged.py tests/test_gpu_dropin.py -q -x $T > gpurun_out/r4_t13_tests.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r4_t13_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base new; do
    L=oac-explore_amd/oac_amd/liboac_amd.so; [ $v = base ] && L=oac-explore_amd/oac_amd/liboac_amd_base.so
    OAC_LIB=$PWD/$L timeout -k 10 200 python tools/launch_times.py --batch 4096 > gpurun_out/r4_t13_lt_$v.log 2>&1; crash $?
    echo "$v $(grep drop-in gpurun_out/r4_t13_lt_$v.log)"; grep 'launch  [0-9] \|launch 1[0-9] ' gpurun_out/r4_t13_lt_$v.log | tr -s ' ' | tr '\n' '|'; echo
    OAC_LIB=$PWD/$L timeout -k 10 200 python tools/launch_times.py --poac --batch 4096 > gpurun_out/r4_t13_ltp_$v.log 2>&1; crash $?
    echo "$v poac $(grep drop-in gpurun_out/r4_t13_ltp_$v.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4_t13_pmc -- python3 $GRAFT_REPO_ROOT/tools/launch_times.py --batch 4096 --steps 10 --rate-steps 50 > $GRAFT_REPO_ROOT/gpurun_out/r4_t13_pmc.log 2>&1; crash $?
echo pmc done
