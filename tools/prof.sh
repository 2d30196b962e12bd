#!/bin/bash
# usage: tools_prof.sh <tag> [bench args...]  -- rocprofv3 kernel trace of a short bench run
set -e
TAG=$1; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -- python3 $R/bench.py --steps 96 --warmup 16 --no-cpu-baseline --no-extras "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
