#!/bin/bash
# kernel traces of the data-parallel drop-in step at one rank over RCCL with
# the exchanges forced: in line, and with the alpha exchange forked onto the
# side stream -- the per-kernel gaps show where the fork / join's time goes
R=$PWD
O=$R/gpurun_out/r6/dpfork
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in inline overlap; do
  F=""; [ $m = overlap ] && F="--overlap"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$m -- python3 $R/tools/dp_trace.py --steps 200 $F > $O/$m.log 2>&1 || exit $?
  python3 $R/tools/dp_trace.py --show $O/$m > $O/${m}_steps.txt || exit $?
  echo "== $m"; cat $O/${m}_steps.txt
done
