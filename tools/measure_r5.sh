#!/bin/bash
# Round-5 measurement session on one MI355X, every figure from the same box:
# the default bench line (the driver's command shape), the B=4096 bench,
# rocprofv3 kernel statistics of the B=256 / B=4096 / configs[4] /
# exploration workloads, the FETCH / WRITE / SQ PMC passes, per-launch
# breakdowns, the exploration stage clocks.  Summaries -> profiles/r05 via
# tools/collect_profiles.sh r05 (run here in the container afterwards).
mkdir -p gpurun_out
R=$PWD
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python bench.py > gpurun_out/bench256.log 2>&1; rc=$?; crash $rc; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/bench256.log | cut -c1-300
timeout -k 10 200 python bench.py --batch 4096 --steps 296 --warmup 32 --no-cpu-baseline --no-extras > gpurun_out/bench4096.log 2>&1; rc=$?; crash $rc; [ $rc -eq 0 ] || exit $rc
bash tools/prof.sh b256; crash $?
bash tools/prof.sh b4096 --batch 4096 --steps 48 --warmup 16; crash $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_poac4096 -- python3 $R/tools/launch_times.py --poac --batch 4096 --steps 8 --rate-steps 200 > $R/gpurun_out/prof_poac4096.log 2>&1); crash $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_expl -- python3 $R/tools/expl_prof.py > $R/gpurun_out/prof_expl.log 2>&1); crash $?
bash tools/pmc.sh b256
bash tools/pmc.sh b4096 --batch 4096
bash tools/pmc_poac.sh
bash tools/pmc_mfma.sh > /dev/null 2>&1
timeout -k 10 200 python tools/launch_times.py --batch 256 > gpurun_out/lt_b256.log 2>&1; crash $?
timeout -k 10 200 python tools/launch_times.py --batch 4096 > gpurun_out/lt_b4096.log 2>&1; crash $?
timeout -k 10 200 python tools/launch_times.py --batch 4096 --poac > gpurun_out/lt_poac.log 2>&1; crash $?
timeout -k 10 60 tools/micro/expl_micro 400 1 0 > gpurun_out/expl_micro.log 2>&1; crash $?
timeout -k 10 120 tools/micro/dataflow_micro > gpurun_out/dataflow_micro.log 2>&1; crash $?
bash tools/pmc_icache.sh > gpurun_out/pmc_icache.txt 2>&1
tail -1 gpurun_out/bench256.log | cut -c1-300
