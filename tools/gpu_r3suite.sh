#!/bin/bash
# the whole GPU suite and smoke() on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
tail -2 gpurun_out/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/suite_smoke.log 2>&1 || { tail -20 gpurun_out/suite_smoke.log; exit 1; }
tail -1 gpurun_out/suite_smoke.log
