"""Helpers for the GPU parity tests: build an oac_amd trainer whose initial
state equals a golden fixture's, and read its gradients / parameters back."""
import numpy as np
import torch
from torch import nn

from fixtures_lib import sac_params, synthetic_transitions


class StateDictModule(nn.Module):
    """What a producer returns: only ``state_dict()`` is read by oac_amd."""

    def __init__(self, sd):
        super().__init__()
        self._sd = sd

    def state_dict(self, *a, **k):
        return {kk: torch.from_numpy(np.ascontiguousarray(v)) for kk, v in self._sd.items()}


class Space:
    def __init__(self, n):
        self.shape = (n,)
        self.low = np.zeros(n, np.float32)


def producers(params, q_keys=("qf1", "qf2", "target_qf1", "target_qf2")):
    it = iter([params[k] for k in q_keys])
    return (lambda **k: StateDictModule(params["policy"]),
            lambda **k: StateDictModule(next(it)))


def sac_trainer_for(meta, params=None, **kw):
    from oac_amd import SACTrainer
    if params is None:
        params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                            pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    pp, qp = producers(params)
    tr = SACTrainer(pp, qp, action_space=Space(meta["act_dim"]), discount=meta["discount"],
                    reward_scale=meta["reward_scale"], policy_lr=meta["lr"], qf_lr=meta["lr"],
                    soft_target_tau=meta["tau"],
                    target_update_period=meta.get("target_update_period", 1),
                    use_automatic_entropy_tuning=meta["auto_alpha"], **kw)
    if meta["auto_alpha"]:
        tr.log_alpha.fill_(meta["log_alpha0"])
    return tr


def module_tensors(tr, mod, arena):
    """{param name: view of ``arena`` (grads / adam_m / ...) at mod's params}."""
    from oac_amd.trainer import _twin_views
    names = [n for n, _ in mod.named_parameters()]
    views = _twin_views(tr.params, arena, [p for _, p in mod.named_parameters()])
    return {n: v for n, v in zip(names, views)}


def batch_from(meta, idx):
    tr = synthetic_transitions(meta["n_replay"], meta["obs_dim"], meta["act_dim"], seed=0)
    return {k: v[idx] for k, v in tr.items()}
