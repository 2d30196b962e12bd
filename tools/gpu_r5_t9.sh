#!/bin/bash
# round 5: per-step device time of the driver-shaped window against the
# warm-up length and an idle gap before the window (clock / cache state)
mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) echo "GPU step ended with $1: stopping"; exit $1;; esac; }
for cfg in "5 0" "100 0" "600 0" "600 20" "5 20"; do
  set -- $cfg
  timeout -k 10 180 python -u tools/fill_drain.py --windows 5 --warmup $1 --idle-ms $2 > gpurun_out/r5_t9_w$1_i$2.txt 2>&1; rc=$?; crash $rc
  python - $1 $2 <<'PY'
import json, sys, numpy as np
rows = [json.loads(l) for l in open(f"gpurun_out/r5_t9_w{sys.argv[1]}_i{sys.argv[2]}.txt") if l.startswith('{"window')]
print("warmup", sys.argv[1], "idle_ms", sys.argv[2], "steps/s", [r["steps_per_s"] for r in rows],
      "first", [r["gpu_step_us"][0] for r in rows], "median step", [float(np.median(r["gpu_step_us"][1:])) for r in rows],
      "fill+drain", [r["fill_plus_drain_us"] for r in rows])
PY
done
