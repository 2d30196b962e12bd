"""Diagnostic: per-tensor gradient error of one SAC step (Humanoid dims) on
the HIP path against the CPU oracle, full tensors, with the location of the
worst elements.  usage: python tools/diag_grads.py [B ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oac-explore_amd")):
    sys.path.insert(0, p)
from fixtures_lib import sac_params, synthetic_transitions  # noqa: E402
from gpu_helpers import Space, module_tensors, producers  # noqa: E402
from oracle import sac_oracle as so  # noqa: E402
import parity  # noqa: E402

HD, HA, HH = 376, 17, 256


def run(B):
    from oac_amd import SACTrainer
    prm = sac_params(HD, HA, [HH, HH], 4, pi_init_w=1e-3, q_init_w=3e-3)
    pp, qp = producers(prm)
    tr = SACTrainer(pp, qp, action_space=Space(HA), discount=0.99, reward_scale=1.0,
                    policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3)
    data = synthetic_transitions(3 * B, HD, HA, seed=0)
    rs = np.random.RandomState(9)
    idx = rs.randint(0, 3 * B, B)
    e1 = rs.standard_normal((B, HA)).astype(np.float32)
    e2 = rs.standard_normal((B, HA)).astype(np.float32)
    batch = {k: v[idx] for k, v in data.items()}
    tr.train_from_torch(batch, eps1=e1, eps2=e2)
    torch.cuda.synchronize()
    orc = so.SACOracle(prm, HD, HA, policy_lr=3e-4, qf_lr=3e-4, tau=5e-3)
    out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
    for grp, mod in (("policy", tr.policy), ("qf1", tr.qf1), ("qf2", tr.qf2)):
        got = module_tensors(tr, mod, tr.grads)
        for name, ref in out["grads"][grp].items():
            g = got[name].cpu().numpy()
            r = ref.numpy()
            e = parity.rel_err(g, r)
            d = np.abs(g - r)
            where = np.unravel_index(np.argsort(d, axis=None)[-4:], d.shape)
            print(f"B={B} {grp:6s} {name:22s} rel {e:.2e}  worst at {list(zip(*where))} "
                  f"got {g[where]} ref {r[where]}", flush=True)


if __name__ == "__main__":
    for b in (sys.argv[1:] or ["4096", "8192"]):
        run(int(b))
