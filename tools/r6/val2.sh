#!/bin/bash
# round 6: the build with the last-arrival Adam in its own kernel instance
# (cur3) against the builds before (sm16) and after (cur2) the variants
O=$PWD/gpurun_out/r6v3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_altkernels.py > $O/alt.txt 2>&1 || { echo "alt tests failed"; tail -30 $O/alt.txt; exit 1; }
tail -1 $O/alt.txt
TAG=val3 VARIANTS="sm16 cur4 cur3" LEGS="b4096 poac" ROUNDS=2 bash tools/r6/ab_libs.sh
