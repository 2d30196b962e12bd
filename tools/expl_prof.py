"""Exploration-call workload for rocprofv3 (profiles/<round>/expl_*): a SAC
trainer at Humanoid dims, then `--reps` single-observation
get_optimistic_exploration_action calls (beta_UB 4.66, delta 23.53) and the
same at 64 observations per call; prints the host wall per call.
usage: python tools/expl_prof.py [--reps N]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--no-cpu-baseline", "--replay", "1000"]
    import bench
    args = bench.parse()
    dev = torch.device("cuda", 0)
    tr, _, _ = bench.build(args, 0, 1, dev)
    out = bench.exploration_timing(tr, args.obs_dim, reps=a.reps)
    print(out, flush=True)


if __name__ == "__main__":
    main()
