#!/bin/bash
# round 5: the library-issued data-parallel step (RCCL hook / gloo callback),
# the BASELINE-dims DP tests, the NaN-head particle test; then the default bench
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_particle.py -v $T -k "split_schedule or nan or rccl_humanoid" -s > gpurun_out/r5_t1_tests.log 2>&1
rc=$?; crash $rc; grep -E "PASS|FAIL|ERROR|dp vs|DP \(|flips" gpurun_out/r5_t1_tests.log | tail -40
timeout -k 10 300 python -u bench.py > gpurun_out/r5_t1_bench.json 2> gpurun_out/r5_t1_bench.err
rc=$?; crash $rc; python -c "
import json; d=json.loads(open('gpurun_out/r5_t1_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'dp1', json.dumps(d.get('dp1'))[:900])"
timeout -k 10 120 tools/micro/bwd_clock_micro 12 12 > gpurun_out/r5_t1_bwd_clock.txt 2>&1; rc=$?; crash $rc; cat gpurun_out/r5_t1_bwd_clock.txt
timeout -k 10 120 tools/micro/fwd_clock_micro > gpurun_out/r5_t1_fwd_clock.txt 2>&1; rc=$?; crash $rc; tail -20 gpurun_out/r5_t1_fwd_clock.txt
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 > gpurun_out/r5_t1_fill.txt 2>&1; rc=$?; crash $rc; tail -7 gpurun_out/r5_t1_fill.txt | cut -c1-400
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 --events 0 > gpurun_out/r5_t1_fill0.txt 2>&1; rc=$?; crash $rc; tail -3 gpurun_out/r5_t1_fill0.txt | cut -c1-300
timeout -k 10 120 tools/micro/dataflow_micro > gpurun_out/r5_t1_dataflow.txt 2>&1; rc=$?; crash $rc; cat gpurun_out/r5_t1_dataflow.txt
CASES="inl:OAC_INLINE_ROWS=1 ring:OAC_INLINE_ROWS=0" timeout -k 10 400 bash tools/ab_b256.sh; rc=$?; crash $rc
for v in 1 0; do OAC_INLINE_ROWS=$v timeout -k 10 120 python tools/launch_times.py > gpurun_out/r5_t1_lt_inl$v.txt 2>&1; rc=$?; crash $rc; head -4 gpurun_out/r5_t1_lt_inl$v.txt | tail -2; done
CASES="devk1:HIP_FORCE_DEV_KERNARG=1 devk0:HIP_FORCE_DEV_KERNARG=0 dflt:X=1" timeout -k 10 600 bash tools/ab_b256.sh; rc=$?; crash $rc
