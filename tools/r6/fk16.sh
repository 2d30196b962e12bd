#!/bin/bash
# round 6: the 16-deep / 4-stage backward ring (cfg 15; the 128x64 form, cfg 16, was measured and removed) -- parity tests,
# then the interleaved micro + step A/B against cfg 12 / 14 (tools/r6/ab2.sh)
O=$PWD/gpurun_out/r6/${TAG:-fk16}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_altkernels.py -k "fk16" > $O/tests.txt 2>&1 || { echo "tests failed: $?"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
TAG=${TAG:-fk16} MICRO="fk:12 fk:15" STEP="fk:12 fk:15" POAC=1 ROUNDS=2 bash tools/r6/ab2.sh
