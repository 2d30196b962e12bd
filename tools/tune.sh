#!/bin/bash
# Small-GEMM geometry sweep: one rocprofv3 kernel trace of a short B=256 bench
# per OAC_TUNE setting ("launch:nw:gpw,..."), per-launch durations of one step.
# usage: tools/tune.sh "<tune string 1>" "<tune string 2>" ...   -> gpurun_out/tune_*.txt
R=$PWD
i=0
for T in "$@"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && OAC_TUNE="$T" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
      -d $R/gpurun_out/tune_$i -- python3 $R/bench.py --steps 64 --warmup 16 --no-cpu-baseline --timing-steps 8 \
      > $R/gpurun_out/tune_$i.log 2>&1 ) || { echo "variant $i failed"; exit 1; }
  echo "== variant $i: OAC_TUNE=$T  $(tail -1 $R/gpurun_out/tune_$i.log | cut -c100-140)" > $R/gpurun_out/tune_$i.txt
  python3 $R/tools/trace.py $R/gpurun_out/tune_$i 13 >> $R/gpurun_out/tune_$i.txt
  rm -rf $R/gpurun_out/tune_$i
  cat $R/gpurun_out/tune_$i.txt
done
