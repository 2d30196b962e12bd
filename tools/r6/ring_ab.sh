#!/bin/bash
# the bench's ring leg (train_from_ring, 64 steps per call) against the drop-in
# line, with and without the next step's critic forward inside the policy
# backward (tuning ring_prefetch); 3 interleaved rounds
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
print(json.dumps(r))
PY
for r in 1 2 3; do
  for t in "" "ring_prefetch=-1"; do
    OAC_TUNE=$t timeout -k 10 200 python /tmp/ring_leg.py > $O/ring_${t:-default}_$r.json 2>$O/ring.err || exit $?
    echo "ring ${t:-default} r$r: $(tail -1 $O/ring_${t:-default}_$r.json)"
  done
done
