"""Does the spread of the sampled replay rows cost the drop-in step?  The
B=256 step with its indices drawn from the first R rows of the 1e6-row
replay (R = 1e6 is the bench's draw) -- the rate over 2,000 steps and the
per-launch durations (dispatch events) of 20, for R in 1e6, 262,144, 65,536,
4,096: the layer-0 launch reads the sampled rows (HBM latency, TLB reach).

Run on the GPU box: python tools/row_locality.py
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


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, rb, _ = bench.build(args, 0, 1, dev)
    from oac_amd import _lib
    L = _lib.lib()
    B = args.batch
    full = rb._size
    np.random.seed(1)
    run = bench.dropin_run(tr, rb, B)
    for rows in (full, 262144, 65536, 4096, full):
        rb._size = rows
        run(200)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(2000)
        torch.cuda.synchronize()
        rate = 2000 / (time.perf_counter() - t0)
        plan = tr._last_plan
        _lib.check(L.oac_sac_set_timing(plan.handle, 1))
        ms = (ctypes.c_double * 4)()
        cnt = (ctypes.c_int64 * 4)()
        _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
        run(20)
        torch.cuda.synchronize()
        cap = 64 * 20
        t = (ctypes.c_double * cap)()
        k = (ctypes.c_int * cap)()
        n = L.oac_sac_read_launch_times(plan.handle, t, k, cap)
        _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
        _lib.check(L.oac_sac_set_timing(plan.handle, 0))
        per = n // 20
        arr = np.median(np.array(t[:per * 20]).reshape(20, per) * 1e3, 0)
        print(f"rows {rows:8d}: {rate:8.1f} steps/s ({1e6 / rate:5.1f} us/step); launches (us): "
              + " ".join(f"{x:.2f}" for x in arr), flush=True)
    rb._size = full


if __name__ == "__main__":
    main()
