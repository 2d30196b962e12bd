"""Break down the host-side latency of one get_optimistic_exploration_action
call (Humanoid dims, one observation): the full call, and its pieces (H2D obs
copy, graph replay + sync, D2H action copy).  usage: python tools/expl_latency.py"""
import os
import sys
import ctypes
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))
import oac_amd  # noqa: E402
from oac_amd import _lib  # noqa: E402
from oac_amd._lib import check, stream_ptr  # noqa: E402


class Space:
    def __init__(self, n):
        self.shape = (n,)


def bench(fn, reps=500):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


def main():
    Do, Da, H = 376, 17, [256, 256]
    dev = torch.device("cuda", 0)
    pp = oac_amd.get_policy_producer(Do, Da, H, device=dev)
    qp = oac_amd.get_q_producer(Do, Da, H, device=dev)
    tr = oac_amd.SACTrainer(pp, qp, action_space=Space(Da), device=dev)
    hp = dict(beta_UB=4.66, delta=23.53, share_layers=False)
    ob = np.random.RandomState(0).standard_normal(Do)
    full = bench(lambda: oac_amd.get_optimistic_exploration_action(ob, policy=tr.policy,
                                                                   qfs=tr.qfs, hyper_params=hp))
    from oac_amd import optimistic_exploration as oe
    oe._USE_GRAPH = True
    full_graph = bench(lambda: oac_amd.get_optimistic_exploration_action(
        ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp))
    oe._USE_GRAPH = False
    e = tr._expl_handle(1)
    L = _lib.lib()
    s = tr.stream
    t_now = bench(lambda: check(L.oac_expl_action_now(e.handle, None, 4.66, 23.53, stream_ptr(s))))
    obs64 = np.random.RandomState(1).standard_normal((64, Do))
    t64 = bench(lambda: oac_amd.get_optimistic_exploration_actions(obs64, policy=tr.policy,
                                                                   qfs=tr.qfs, hyper_params=hp))

    def launch():
        check(L.oac_expl_action(e.handle, None, 4.66, 23.53, None, None, None, None,
                                stream_ptr(s)))
        s.synchronize()
    t_launch = bench(launch)
    z = torch.zeros(1, device=dev)

    def tiny():
        with torch.cuda.stream(s):
            z.add_(1.0)
        s.synchronize()
    t_tiny = bench(tiny)
    po, pr = ctypes.c_void_p(), ctypes.c_void_p()
    check(L.oac_expl_set_host_io(e.handle, None, None))   # device-only graph
    t_kernel = bench(launch)
    check(L.oac_expl_host_staging(e.handle, ctypes.byref(po), ctypes.byref(pr)))
    check(L.oac_expl_set_host_io(e.handle, po, pr))
    print({"full_call_us": round(full, 1), "full_call_graph_us": round(full_graph, 1),
           "action_now_us": round(t_now, 1), "call_64obs_us": round(t64, 1), "graph_with_host_io_sync_us": round(t_launch, 1),
           "graph_device_only_sync_us": round(t_kernel, 1),
           "tiny_kernel_sync_us": round(t_tiny, 1)})


if __name__ == "__main__":
    main()
