"""The data-parallel drop-in step at one rank over RCCL with the exchanges
forced (bench.py's dp1 `with_rccl_allreduces` leg), for a kernel trace:
run under rocprofv3 --kernel-trace, then `python tools/dp_trace.py --show DIR`
prints one step's kernels (every kernel, RCCL's included) with durations and
the gap before each.

usage: rocprofv3 --kernel-trace --output-format csv -d DIR -- python tools/dp_trace.py [--steps N]
       python tools/dp_trace.py --show DIR"""
import argparse
import csv
import datetime
import glob
import os
import sys


def show(d):
    f = max(glob.glob(d + "/*/*_kernel_trace.csv"), key=os.path.getmtime)
    r = list(csv.DictReader(open(f)))
    r.sort(key=lambda x: int(x["Start_Timestamp"]))
    # a step starts at the layer-0 launch: the small kernel's inline-rows form
    starts = [i for i, x in enumerate(r) if "gemm_small_kernel_inl" in x["Kernel_Name"]]
    if len(starts) < 4:
        sys.exit("too few steps in the trace")
    mid = len(starts) // 2
    for a, b in ((starts[mid], starts[mid + 1]), (starts[mid + 1], starts[mid + 2])):
        t_prev = None
        tot = 0.0
        for x in r[a:b]:
            s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
            gap = (s - t_prev) / 1e3 if t_prev is not None else 0.0
            tot += (e - s) / 1e3
            print(f"  {(e - s) / 1e3:7.2f} us  gap {gap:6.2f}  {x['Kernel_Name'][:90]}")
            t_prev = e
        span = (int(r[b]["Start_Timestamp"]) - int(r[a]["Start_Timestamp"])) / 1e3
        print(f"step: {b - a} kernels, kernel sum {tot:.1f} us, start-to-next-start {span:.1f} us\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--show", default=None)
    ap.add_argument("--overlap", action="store_true",
                    help="the alpha exchange on the side stream (force_overlap)")
    a = ap.parse_args()
    if a.show:
        show(a.show)
        return
    import numpy as np
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oac-explore_amd")]
    sys.argv = [sys.argv[0]]
    import bench
    import oac_amd
    from oac_amd.dp import DataParallelSACTrainer
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _, rb, _ = bench.build(args, 0, 1, dev)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(bench._free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                            timeout=datetime.timedelta(seconds=120))
    try:
        torch.manual_seed(0)
        hid = [args.hidden, args.hidden]
        pp = oac_amd.get_policy_producer(args.obs_dim, args.act_dim, hid, device=dev)
        qp = oac_amd.get_q_producer(args.obs_dim, args.act_dim, hid, device=dev)
        with DataParallelSACTrainer(pp, qp, action_space=bench.Space(args.act_dim), discount=0.99,
                                    reward_scale=1.0, policy_lr=3e-4, qf_lr=3e-4,
                                    soft_target_tau=5e-3, target_update_period=1,
                                    use_automatic_entropy_tuning=True, device=dev, seed=2,
                                    force_collectives=True, force_overlap=a.overlap) as tr:
            np.random.seed(1)
            run = bench.dropin_run(tr, rb, args.batch)
            run(a.steps)
            torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
