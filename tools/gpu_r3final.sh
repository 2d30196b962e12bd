#!/bin/bash
# round-3 final: the whole GPU suite, smoke(), then tools/measure_r3.sh (bench, rocprof, PMC, per-launch)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_gputests.log 2>&1 || { tail -40 gpurun_out/final_gputests.log; exit 1; }
tail -2 gpurun_out/final_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/measure_r3.sh
