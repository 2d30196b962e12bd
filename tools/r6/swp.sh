#!/bin/bash
# round 6: the software-pipelined backward loop (cfg 17 / 18) -- parity tests,
# stage clocks, then the interleaved micro + step A/B against cfg 12 / 14
O=$PWD/gpurun_out/r6/${TAG:-swp2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_altkernels.py -k "swp" > $O/tests.txt 2>&1 || { echo "tests failed: $?"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for c in 12 17; do
  timeout -k 5 60 tools/micro/bwd_clock_micro $c 1 > $O/clock_$c.txt 2>&1 || exit $?
done
TAG=${TAG:-swp2} MICRO="fk:12 fk:17" STEP="fk:12 fk:17" POAC=1 ROUNDS=3 bash tools/r6/ab2.sh
