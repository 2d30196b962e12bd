#!/bin/bash
# round 5: the library-issued data-parallel step (RCCL hook / gloo callback),
# the BASELINE-dims DP tests, the NaN-head particle test; then the default bench
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
T="--timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_particle.py -v -x $T > gpurun_out/r5_t1_tests.log 2>&1
rc=$?; crash $rc; grep -E "PASS|FAIL|ERROR|dp vs|DP \(" gpurun_out/r5_t1_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5_t1_bench.json 2> gpurun_out/r5_t1_bench.err
rc=$?; crash $rc; python -c "
import json; d=json.loads(open('gpurun_out/r5_t1_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'dp1', json.dumps(d.get('dp1'))[:900])"
