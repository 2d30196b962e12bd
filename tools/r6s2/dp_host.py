"""Host issue time against completion time per drop-in step, single process
against the data-parallel step at one rank with the three RCCL all-reduces
forced (bench.py's dp1 leg): is the DP step host-bound?
Run on the GPU box: python tools/r6s2/dp_host.py"""
import datetime
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))
sys.argv = [sys.argv[0], "--no-cpu-baseline"]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def measure(tr, rb, B, K=400, burst=8, bursts=50):
    """(host issue us/step of K steps in a row -- throttled by the index
    ring's chunk events once it is 16 slots ahead --, completion us/step,
    host issue us/step of `burst`-step bursts after a sync -- the host's own
    cost, nothing to wait on --, median over `bursts`)"""
    run = bench.dropin_run(tr, rb, B)
    np.random.seed(1)
    run(64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(K)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    bs = []
    for _ in range(bursts):
        torch.cuda.synchronize()
        a = time.perf_counter()
        run(burst)
        bs.append(1e6 * (time.perf_counter() - a) / burst)
    torch.cuda.synchronize()
    return 1e6 * (t1 - t0) / K, 1e6 * (t2 - t0) / K, float(np.median(bs))


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, rb, _ = bench.build(args, 0, 1, dev)
    B = args.batch
    for r in range(2):
        h, t, hb = measure(tr, rb, B)
        print(f"single   host issue {h:6.1f} us/step  completion {t:6.1f} us/step  "
              f"host issue in 8-step bursts {hb:6.1f} us/step", flush=True)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(bench._free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                            timeout=datetime.timedelta(seconds=120))
    import oac_amd
    from oac_amd.dp import DataParallelSACTrainer
    hid = [args.hidden, args.hidden]
    pp = oac_amd.get_policy_producer(args.obs_dim, args.act_dim, hid, device=dev)
    qp = oac_amd.get_q_producer(args.obs_dim, args.act_dim, hid, device=dev)
    with DataParallelSACTrainer(pp, qp, action_space=bench.Space(args.act_dim), discount=0.99,
                                reward_scale=1.0, policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3,
                                target_update_period=1, use_automatic_entropy_tuning=True,
                                device=dev, seed=2, force_collectives=True) as dtr:
        for r in range(2):
            h, t, hb = measure(dtr, rb, B)
            print(f"dp+rccl  host issue {h:6.1f} us/step  completion {t:6.1f} us/step  "
                  f"host issue in 8-step bursts {hb:6.1f} us/step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
