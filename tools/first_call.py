"""Host time of the first drop-in step after the device went idle (the
driver's timed window starts right after a synchronize): per call part --
random_batch, train() -- for the first and the following calls, and the same
for a bare torch launch and a bare library call, to see where the first
call's extra time goes.

Run on the GPU box: python tools/first_call.py
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oac-explore_amd")]
import bench  # noqa: E402


def us(t):
    return round(t * 1e6, 1)


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    tr, rb, _ = bench.build(args, 0, 1, device)
    from oac_amd import _lib
    L = _lib.lib()
    B = args.batch
    np.random.seed(1)
    for _ in range(30):
        d = rb.random_batch(B)
        tr.train(d)
    x = torch.zeros(16, device=device)
    rows = []
    for trial in range(6):
        for idle in (0.0, 0.002):
            torch.cuda.synchronize()
            if idle:
                time.sleep(idle)
            t = [time.perf_counter()]
            d = rb.random_batch(B)
            t.append(time.perf_counter())
            tr.train(d)
            t.append(time.perf_counter())
            d = rb.random_batch(B)
            t.append(time.perf_counter())
            tr.train(d)
            t.append(time.perf_counter())
            torch.cuda.synchronize()
            # a bare torch kernel launch after idle, then a second one
            t2 = [time.perf_counter()]
            x.add_(1.0)
            t2.append(time.perf_counter())
            x.add_(1.0)
            t2.append(time.perf_counter())
            torch.cuda.synchronize()
            # a library call that launches nothing
            t3 = time.perf_counter()
            L.oac_sac_launch_count(tr._last_plan.handle)
            t4 = time.perf_counter()
            rows.append(dict(idle_s=idle, random_batch_1=us(t[1] - t[0]), train_1=us(t[2] - t[1]),
                             random_batch_2=us(t[3] - t[2]), train_2=us(t[4] - t[3]),
                             torch_launch_1=us(t2[1] - t2[0]), torch_launch_2=us(t2[2] - t2[1]),
                             lib_noop=us(t4 - t3)))
            print(rows[-1], flush=True)
    # per-launch host cost inside the first train() after idle: the step's
    # launches issued with the plan's timing off, timed around the ctypes call
    print("median first / second train():",
          np.median([r["train_1"] for r in rows]), np.median([r["train_2"] for r in rows]))


if __name__ == "__main__":
    main()
