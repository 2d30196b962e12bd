#!/bin/bash
# the B=256 step's per-edge trace with the step as one graph launch (same
# kernels; under rocprofv3 the direct-launch drop-in is host-bound, so its
# kernels start after host gaps and the trace shows no back-to-back steps)
mkdir -p gpurun_out
OAC_DROPIN_GRAPH=1 bash tools/prof.sh b256g; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 tools/trace.py gpurun_out/prof_b256g 11 | tail -3
