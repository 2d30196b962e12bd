"""Run by tests/test_gpu_altkernels.py in child processes: three large-batch
steps (B = 1100, hidden 48 / 80) of SACTrainer and ParticleTrainerOAC with
fixed batches and eps; the trainers' params / targets / Adam moments are
written to the .npz path given on the command line.  The parent compares the
side-workgroup Adam (tuning split_adam, the SAC step) against one Adam
launch per group: the same adam_flat_elem on the same slabs, so bit for bit."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oac-explore_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fixtures_lib import sac_params  # noqa: E402
from gpu_helpers import Space, producers  # noqa: E402
import test_gpu_ragged as tr  # noqa: E402
from oac_amd import _lib  # noqa: E402

# the kernel / schedule choice of this child (oac_tuning_set), from the parent
_lib.set_tuning_spec(os.environ.get("OAC_TEST_TUNING", ""))


def _run(trainer, Do, Da, B, seed):
    rs = np.random.RandomState(seed)
    for step in range(3):
        b = tr._batch(Do, Da, B, seed + step)
        e1 = rs.standard_normal((B, Da)).astype(np.float32)
        e2 = rs.standard_normal((B, Da)).astype(np.float32)
        trainer.train_from_torch(b, eps1=e1, eps2=e2)
    torch.cuda.synchronize()
    return {k: getattr(trainer, k).cpu().numpy() for k in ("params", "targets", "adam_m", "adam_v")}


def main(out):
    from oac_amd import ParticleTrainerOAC, SACTrainer
    res, trace = {}, {}
    for Do, Da, H, B in [(7, 5, 48, 1100), (13, 6, 80, 1029)]:
        pp, qp = producers(sac_params(Do, Da, [H, H], 3, pi_init_w=0.2, q_init_w=0.1))
        sac = SACTrainer(pp, qp, action_space=Space(Da), policy_lr=3e-4, qf_lr=3e-4,
                         soft_target_tau=5e-3, use_automatic_entropy_tuning=True)
        for k, v in _run(sac, Do, Da, B, 11).items():
            res[f"sac_{H}_{k}"] = v
        # the step's trace bits (not compared: the parent checks the path taken)
        trace[f"sac_{H}"] = _lib.lib().oac_sac_trace(sac._last_plan.handle, 1)
        K = 7
        pp, qp = producers(sac_params(Do, Da, [H, H], 3, q_out=K, pi_init_w=0.2, q_init_w=0.1,
                                      q_last_bias=np.linspace(0.0, 30.0, K)),
                           q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1", "target_qf1"))
        poac = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), policy_lr=3e-4,
                                  qf_lr=3e-4, soft_target_tau=5e-3,
                                  use_automatic_entropy_tuning=True, deterministic=False,
                                  q_min=0.0, q_max=30.0, share_layers=True)
        for k, v in _run(poac, Do, Da, B, 21).items():
            res[f"poac_{H}_{k}"] = v
    np.savez(out, **res)
    print("ok", len(res), "trace", " ".join(f"{k}={v}" for k, v in sorted(trace.items())), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
