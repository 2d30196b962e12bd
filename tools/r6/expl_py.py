"""Where the Python exploration call's time goes on top of the library call
(round 6): the full get_optimistic_exploration_action, the same call with
its library call replaced by a no-op (the Python path alone), and the bare
library call with its arguments prepared once.
usage (GPU box): python tools/r6/expl_py.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oac-explore_amd"), os.path.join(ROOT, "tests")]
import oac_amd  # noqa: E402
from oac_amd import _lib, get_optimistic_exploration_action  # noqa: E402
from oac_amd import optimistic_exploration as oe  # noqa: E402
from gpu_helpers import Space  # noqa: E402


def timeit(fn, reps=400, runs=5):
    for _ in range(50):
        fn()
    out = []
    for _ in range(runs):
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        out.append(1e6 * (time.perf_counter() - t0) / reps)
    return float(np.median(out))


def main():
    dev = torch.device("cuda", 0)
    Do, Da = 376, 17
    pp = oac_amd.get_policy_producer(Do, Da, [256, 256], device=dev)
    qp = oac_amd.get_q_producer(Do, Da, [256, 256], device=dev)
    tr = oac_amd.SACTrainer(pp, qp, action_space=Space(Da))
    hp = dict(beta_UB=4.66, delta=23.53, share_layers=False)
    ob = np.random.RandomState(0).standard_normal(Do)
    full = timeit(lambda: get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs,
                                                            hyper_params=hp))
    L = _lib.lib()
    e = tr._expl_handle(1)
    s = ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(0))
    fn = L.oac_expl_action_now
    bare = timeit(lambda: fn(e.handle, None, 4.66, 23.53, s))

    class NoLib:   # the Python path with the library call a no-op
        def __getattr__(self, k):
            return (lambda *a: 0) if k.startswith("oac_expl") else getattr(L, k)
    real = _lib.lib
    _lib.lib = lambda: NoLib()
    tr.policy.__dict__.pop(oe._CACHE_ATTR, None)   # (the cached call record holds the library)
    try:
        py = timeit(lambda: get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs,
                                                              hyper_params=hp))
    finally:
        _lib.lib = real
        tr.policy.__dict__.pop(oe._CACHE_ATTR, None)
    print(f"full call {full:.2f} us; bare library call {bare:.2f} us; Python path alone {py:.2f} us")


if __name__ == "__main__":
    main()
