#!/bin/bash
# the GPU test suite (or the files given as arguments), one process, bounded
O=$PWD/gpurun_out/r6
mkdir -p $O
T=${1:-tests}
shift
timeout -k 10 ${TLIM:-1100} python -u -m pytest $T "$@" -m gpu -x -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > $O/gputests_${TAG:-all}.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/gputests_${TAG:-all}.log | tail -3
exit $rc
