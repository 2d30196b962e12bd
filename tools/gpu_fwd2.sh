#!/bin/bash
# cfg-6 forward kernel: large-batch parity tests with it on, then B=4096 launch times for both tiles
mkdir -p gpurun_out
OAC_FWD2=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "4096 or b4096 or poac or particle or goac or ptrain or dp" > gpurun_out/pytest_fwd2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fwd2.log; grep -E "^FAILED|Error" gpurun_out/pytest_fwd2.log | head -5; [ $rc -eq 0 ] || exit $rc
for tile in 128 64; do
  echo "tile $tile"; OAC_FWD2=1 OAC_FWD2_TILE=$tile timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 > gpurun_out/lt_fwd2_$tile.txt || exit 1
  grep -E "B=|launch ( 1| 2| 5)" gpurun_out/lt_fwd2_$tile.txt
done
timeout -k 10 200 python tools/launch_times.py --batch 4096 --rate-steps 500 | grep -E "B=|launch ( 1| 2| 5) "
