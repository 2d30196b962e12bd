#!/bin/bash
# the bench's ring leg (train_from_ring, 64 steps per call) against the drop-in
# loop on the same trainer: the ring step's default form (rows through the
# device index ring), the gather launch per 8 steps (ring_direct=-1), and that
# with the next step's critic forward inside the policy backward
# (ring_prefetch=1); 3 interleaved rounds
O=$PWD/gpurun_out/r6/ring
mkdir -p $O
cat > /tmp/ring_leg.py <<'PY'
import json, os, sys
sys.argv = [sys.argv[0], "--no-cpu-baseline"]
sys.path.insert(0, os.getcwd())
import bench, torch
from oac_amd import _lib
_lib.set_tuning_spec(os.environ.get("OAC_TUNE", ""))
args = bench.parse()
dev = torch.device("cuda", 0)
tr, rb, stream = bench.build(args, 0, 1, dev)
r = bench.ring_timing(tr, stream, rb, 256, steps=1280)
run = bench.dropin_run(tr, rb, 256)
import time, numpy as np
np.random.seed(1)
run(200); torch.cuda.synchronize()
t0 = time.perf_counter(); run(1280); torch.cuda.synchronize()
r["dropin_steps_per_s"] = round(1280 / (time.perf_counter() - t0), 1)
print(json.dumps(r))
PY
for r in 1 2 3; do
  for t in "" "ring_direct=-1" "ring_direct=-1,ring_prefetch=1"; do
    OAC_TUNE=$t timeout -k 10 200 python /tmp/ring_leg.py > $O/ring_${t:-default}_$r.json 2>$O/ring.err || exit $?
    echo "ring ${t:-default} r$r: $(tail -1 $O/ring_${t:-default}_$r.json)"
  done
done
