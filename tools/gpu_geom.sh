#!/bin/bash
# LDS kernel tile variants at B=4096: large-batch parity per variant, then the step's launch times
mkdir -p gpurun_out
for g in 0 1 2 3; do
  OAC_LDS_GEOM=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_particle.py tests/test_gpu_ragged.py -x -q -k "4096 or 1024 or ragged" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_geom$g.log 2>&1 || { echo "geom $g FAILED"; tail -20 gpurun_out/pytest_geom$g.log; exit 1; }
  echo "geom $g: $(tail -1 gpurun_out/pytest_geom$g.log)"
  OAC_LDS_GEOM=$g timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 300 2>&1 | grep -v amdgpu.ids | head -1
done
OAC_LDS2=0 timeout -k 10 200 python tools/launch_times.py --batch 4096 --steps 10 --rate-steps 300 2>&1 | grep -v amdgpu.ids | head -1
