#!/bin/bash
# Round measurement on one MI355X: bench lines (B=256 headline, B=4096), the
# rocprofv3 kernel-trace stats of both, and the FETCH/WRITE/SQ PMC passes
# (FETCH/WRITE also over the configs[4] P-OAC workload).
# Outputs under gpurun_out/; copy the summaries into profiles/<round>/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench256.log 2>&1 &&
timeout -k 10 200 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline > gpurun_out/bench4096.log 2>&1 &&
bash tools/prof.sh b256 &&
bash tools/prof.sh b4096 --batch 4096 --steps 48 --warmup 16 &&
bash tools/pmc.sh b256 &&
bash tools/pmc.sh b4096 --batch 4096 &&
bash tools/pmc_poac.sh
rc=$?
tail -1 gpurun_out/bench256.log | cut -c1-400
exit $rc
