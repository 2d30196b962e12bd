"""Where the driver-shaped bench window goes (bench.py --steps 20 --warmup 5):
per-step GPU intervals from events recorded between the drop-in steps, the
host's issue times, and the window's fill (t0 -> first event) and drain
(last event -> synchronize returns), for several windows on one trainer.

Run on the GPU box: python tools/fill_drain.py [--windows 8] [--steps 20]
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oac-explore_amd")]
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--events", type=int, default=1, help="record an event between steps")
    ap.add_argument("--idle-ms", type=float, default=0.0,
                    help="host sleep between the warm-up's synchronize and the window")
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    tr, rb, _ = bench.build(args, 0, 1, device)
    B = args.batch
    np.random.seed(1)

    def step():
        d = rb.random_batch(B)
        d["buffer"] = rb
        tr.train(d)

    out = []
    for w in range(a.windows):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
        for e in evs:   # torch creates the HIP event on its first record: not inside the window
            e.record()
        host = []
        gc.collect()    # (before the warm-up, as bench.py: it leaves the host caches cold)
        gc.disable()
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        if a.idle_ms:
            time.sleep(a.idle_ms * 1e-3)
        t0 = time.perf_counter()
        if a.events:
            evs[0].record()
        for i in range(a.steps):
            step()
            host.append(time.perf_counter() - t0)
            if a.events:
                evs[i + 1].record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        gc.enable()
        rec = {"window_us": round(el * 1e6, 1), "steps_per_s": round(a.steps / el, 1),
               "host_issue_us": [round(h * 1e6, 1) for h in host]}
        if a.events:
            gpu = [evs[0].elapsed_time(evs[i + 1]) * 1e3 for i in range(a.steps)]
            per = np.diff([0.0] + gpu)
            rec["gpu_step_us"] = [round(x, 1) for x in per]
            rec["gpu_span_us"] = round(gpu[-1], 1)
            rec["fill_plus_drain_us"] = round(el * 1e6 - gpu[-1], 1)
        out.append(rec)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"median_steps_per_s": float(np.median([r["steps_per_s"] for r in out]))}))


if __name__ == "__main__":
    main()
