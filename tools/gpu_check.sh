#!/bin/bash
# One GPU round trip: parity tests, B=256 / B=4096 bench lines, and a
# per-launch kernel trace of the B=256 step (rocprofv3).  Outputs under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --steps-per-launch 1 > gpurun_out/bench256_spl1.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline > gpurun_out/bench256.log 2>&1 &&
timeout -k 10 200 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline > gpurun_out/bench4096.log 2>&1 &&
bash tools/prof.sh b256 &&
python tools/trace.py gpurun_out/prof_b256 ${NLAUNCH:-19} > gpurun_out/trace_b256.txt
rc=$?
tail -1 gpurun_out/bench256_spl1.log | cut -c1-330
tail -1 gpurun_out/bench256.log | cut -c1-330
tail -1 gpurun_out/bench4096.log | cut -c1-330
cat gpurun_out/trace_b256.txt
exit $rc
