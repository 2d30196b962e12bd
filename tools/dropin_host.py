"""Host-side cost of the drop-in call pattern (rl_algorithm.py:160-167):
where the microseconds of one random_batch + train call go."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0], "--no-cpu-baseline"]
import bench  # noqa: E402
from oac_amd import _lib  # noqa: E402

args = bench.parse()
dev = torch.device("cuda", 0)
tr, rb, st = bench.build(args, 0, 1, dev)
B = args.batch
np.random.seed(1)
for _ in range(50):
    b = rb.random_batch(B)
    tr.train(b)
torch.cuda.synchronize()


def t(fn, n=2000):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return 1e6 * (time.perf_counter() - t0) / n


res = {}
res["np_randint"] = t(lambda: np.random.randint(0, 1_000_000, B))
res["random_batch"] = t(lambda: rb.random_batch(B))
batches = [rb.random_batch(B) for _ in range(2000)]
it = iter(batches)
torch.cuda.synchronize()
res["train_call"] = t(lambda: tr.train(next(it)), n=100)
torch.cuda.synchronize()
plan = tr._last_plan
L = _lib.lib()
idx = np.random.randint(0, 1_000_000, B)
sp = _lib.stream_ptr(torch.cuda.current_stream(dev))
p = ctypes.c_void_p(idx.ctypes.data)


def raw():
    _lib.check(L.oac_sac_step_host_idx(plan.handle, p, tr._bc_mirror, _lib.OAC_STEP_DEVICE_EPS, sp))
    tr._bc_mirror += 1


res["raw_c_step"] = t(raw, n=100)
torch.cuda.synchronize()
res["stream_ptr"] = t(lambda: _lib.stream_ptr(torch.cuda.current_stream(dev)))
print({k: round(v, 2) for k, v in res.items()})
