"""Per-launch device durations of the drop-in step (direct launches with
hipExtLaunchKernel start/stop events; the same kernels the step's graph
runs), averaged over n steps, plus the drop-in step rate with graphs.
usage: python tools/launch_times.py [--batch B] [--steps N]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rate-steps", type=int, default=2000)
    ap.add_argument("--poac", action="store_true",
                    help="BASELINE configs[4]: ParticleTrainerOAC K=10, Ant dims")
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--no-cpu-baseline", "--batch", str(a.batch)]
    import bench
    from oac_amd import _lib
    # OAC_TUNE="key=value,...": non-default kernel choices (oac_tuning_set)
    if hasattr(_lib.lib(), "oac_tuning_set"):   # (older A/B builds read OAC_* env switches)
        _lib.set_tuning_spec(os.environ.get("OAC_TUNE", ""))
    args = bench.parse()
    dev = torch.device("cuda", 0)
    if a.poac:   # the trainer and replay of bench.poac_ant_leg
        import oac_amd
        Do, Da, K = 111, 8, 10
        torch.manual_seed(0)
        pp = oac_amd.get_policy_producer(Do, Da, [256, 256], device=dev)
        qp = oac_amd.get_q_producer(Do, Da, [256, 256], output_size=K, device=dev)
        tr = oac_amd.ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=bench.Space(Da),
                                        discount=0.99, policy_lr=3e-4, qf_lr=3e-4,
                                        soft_target_tau=5e-3, use_automatic_entropy_tuning=True,
                                        deterministic=False, q_min=0.0, q_max=500.0,
                                        share_layers=True, device=dev)
        rb = oac_amd.ReplayBuffer(args.replay, Do, Da, device=dev)
        rb.load_transitions(bench.synthetic_rows(args.replay, rb.rows, Do, Da, dev, seed=3))
    else:
        tr, rb, _ = bench.build(args, 0, 1, dev)
    B = a.batch
    np.random.seed(1)
    run = bench.dropin_run(tr, rb, B)
    run(200)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.rate_steps)
    torch.cuda.synchronize()
    rate = a.rate_steps / (time.perf_counter() - t0)
    plan = tr._last_plan
    L = _lib.lib()
    _lib.check(L.oac_sac_set_timing(plan.handle, 1))
    ms = (ctypes.c_double * 4)()
    cnt = (ctypes.c_int64 * 4)()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
    run(a.steps)
    torch.cuda.synchronize()
    cap = 64 * a.steps
    t = (ctypes.c_double * cap)()
    k = (ctypes.c_int * cap)()
    n = L.oac_sac_read_launch_times(plan.handle, t, k, cap)
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
    _lib.check(L.oac_sac_set_timing(plan.handle, 0))
    per = n // a.steps
    arr = np.array(t[:n]).reshape(a.steps, per) * 1e3
    kinds = list(k[:per])
    names = ["gemm", "row", "adam", "gather"]
    print(f"B={B}: drop-in {rate:.1f} steps/s ({1e6 / rate:.1f} us/step); {per} launches/step, "
          f"sum of launch durations {arr.mean(0).sum():.1f} us")
    for i in range(per):
        print(f"  launch {i:2d} {names[kinds[i]]:6s} {np.median(arr[:, i]):7.2f} us")


if __name__ == "__main__":
    main()
