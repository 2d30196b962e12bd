#!/bin/bash
# round 5: the inline-index layer-0 launch read in place (no scratch copy);
# drop-in parity, the DP tests at BASELINE dims, A/B and the first-call probe
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_ring.py -q -x $T > gpurun_out/r5_t3_dropin.log 2>&1
rc=$?; crash $rc; tail -2 gpurun_out/r5_t3_dropin.log; [ $rc -eq 0 ] || exit $rc
CASES="inl:OAC_INLINE_ROWS=1 ring:OAC_INLINE_ROWS=0" timeout -k 10 400 bash tools/ab_b256.sh; rc=$?; crash $rc
for v in 1 0; do OAC_INLINE_ROWS=$v timeout -k 10 120 python tools/launch_times.py > gpurun_out/r5_t3_lt_inl$v.txt 2>&1; rc=$?; crash $rc; head -4 gpurun_out/r5_t3_lt_inl$v.txt | tail -3; done
timeout -k 10 120 python -u tools/first_call.py > gpurun_out/r5_t3_first.txt 2>&1; rc=$?; crash $rc; cat gpurun_out/r5_t3_first.txt | tail -14
echo skip-dp
rc=$?; crash $rc; grep -E "PASS|FAIL|ERROR|dp vs|DP \(|flips" gpurun_out/r5_t3_dp.log | tail -20
timeout -k 10 180 python -u tools/fill_drain.py --windows 6 > gpurun_out/r5_t3_fill.txt 2>&1; rc=$?; crash $rc; tail -7 gpurun_out/r5_t3_fill.txt | cut -c1-600
