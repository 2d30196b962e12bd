"""The data-parallel drop-in step at one rank over RCCL against the
single-process drop-in step, same replay and loop (bench.py's dp1 leg alone).
Run on the GPU box: python tools/dp1_ab.py [--batch B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse()
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    tr, rb, _ = bench.build(args, 0, 1, device)
    B = args.batch
    np.random.seed(1)
    el = bench.timed(bench.dropin_run(tr, rb, B), args.steps, args.warmup, 1, device)
    single = args.steps / el
    out = {"batch": B, "single_steps_per_s": round(single, 1),
           "dp1": bench.dp1_leg(args, rb, device, B, single, steps=args.steps,
                                warmup=args.warmup)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
