"""Host vs device time of the bench's ring-step calls: issue time of K calls
(no sync) against their completion time, and the device time of the same
calls measured with torch events on the trainer's stream."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--no-cpu-baseline"]
import bench  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
tr, rb, st = bench.build(args, 0, 1, dev)
n = 8
step = bench.step_fn(tr, rb, st, args.batch, n)
for _ in range(10):
    step()
torch.cuda.synchronize()
K = 40
t0 = time.perf_counter()
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
e0.record(tr.stream)
for _ in range(K):
    step()
t_issue = time.perf_counter() - t0
e1.record(tr.stream)
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"{K} calls x {n} steps: host issue {1e6 * t_issue / K:.1f} us/call, wall {1e6 * t_all / K:.1f} us/call, "
      f"device (events on trainer stream) {1e3 * e0.elapsed_time(e1) / K:.1f} us/call")
