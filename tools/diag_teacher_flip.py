"""Where a teacher-forced step's policy-gradient mismatch comes from: per step
of a SAC fixture (GPU state loaded into the oracle as in
tests/test_gpu_teacher.py), the policy gradient errors per parameter, how many
fc0 rows carry the error, and the closest-to-0 pre-activations (|pre| / rms)
of the policy trunk and of both critics' policy-loss passes, and the closest
q1 / q2 near-tie of the min.

Run on the GPU box: python tools/diag_teacher_flip.py [fixture]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oac-explore_amd")]
import parity  # noqa: E402
from gpu_helpers import batch_from, module_tensors  # noqa: E402
from gpu_helpers import sac_trainer_for  # noqa: E402
from oracle import sac_oracle as so  # noqa: E402
from test_gpu_teacher import sac_oracle_from_gpu  # noqa: E402


def near0(hs, p):
    out = []
    for i in range(len(hs) - 1):
        W = p[f"fc{i}.weight"].double()
        b = p[f"fc{i}.bias"].double()
        pre = hs[i].double() @ W.t() + b
        rms = pre.pow(2).mean().sqrt()
        a = (pre.abs() / rms)
        out.append(float(a.min()))
    return out


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "sac_humanoid_b4096"
    meta, g = parity.load(name)
    tr = sac_trainer_for(meta)
    for s in range(meta["steps"]):
        orc = sac_oracle_from_gpu(tr, meta)
        batch = batch_from(meta, g[f"s{s}/idx"])
        e1, e2 = g[f"s{s}/eps1"], g[f"s{s}/eps2"]
        tr.end_epoch(s)
        tr.train_from_torch(batch, eps1=e1, eps2=e2)
        torch.cuda.synchronize()
        out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
        gv = module_tensors(tr, tr.policy, tr.grads)
        rec = {"step": s}
        for pn, ref in out["grads"]["policy"].items():
            got = gv[pn].cpu().numpy()
            rec[pn] = float(parity.rel_err(got, ref.numpy()))
        d = np.abs(gv["fc0.weight"].cpu().numpy() - out["grads"]["policy"]["fc0.weight"].numpy())
        rd = d.max(axis=1)
        rec["fc0_rows_err_gt_1pct_max"] = int((rd > 0.01 * rd.max()).sum()) if rd.max() > 0 else 0
        S = orc.S
        rec["policy_near0"] = near0(S["pf"]["hs"], orc.P)
        rec["c1n_near0"] = near0(S["c1n"]["hs"], orc.Q1)
        rec["c2n_near0"] = near0(S["c2n"]["hs"], orc.Q2)
        q1, q2 = S["c1n"]["q"].double(), S["c2n"]["q"].double()
        rec["min_tie"] = float(((q1 - q2).abs() / q1.abs().mean()).min())
        ls = S["pf"]["ls_raw"].double()
        rec["logstd_clamp_dist"] = float(torch.minimum((ls - so.LOG_SIG_MIN).abs(),
                                                       (ls - so.LOG_SIG_MAX).abs()).min())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
