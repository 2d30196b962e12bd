#!/bin/bash
# exploration: parity tests, then the latency breakdown and a kernel trace
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "expl or exploration" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_expl.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_expl.log; grep -E "^FAILED|Error" gpurun_out/pytest_expl.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/expl_latency.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/expl_prof -o run -- python3 tools/expl_latency.py > gpurun_out/expl_prof.log 2>&1 || exit 1
f=$(find gpurun_out/expl_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-6 "$f" | grep -i expl
