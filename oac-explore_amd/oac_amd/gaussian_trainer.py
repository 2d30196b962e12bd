"""Drop-in ``GaussianTrainer`` of the g-oac recipes
(/root/reference/trainer/gaussian_trainer.py:14-538, the trainer main.py
builds for ``--alg g-oac``, main.py:219-233), in the configuration every
reproduce_g-oac*.sh recipe runs: ``--share_layers`` (one critic with two
outputs, Q mean | log std, exp'd by ``positive=[False, True]``), the
deterministic policy (GaussianTrainer's default, not overridden for g-oac),
optionally ``--counts`` / ``std_soft_update`` / ``--mean_update``.  The step
runs in liboac_amd (csrc/det_plan.hip); the interface is the reference's:
constructor kwargs, ``train`` / ``train_from_torch``, ``predict``,
``obj_func``, ``get_diagnostics``, ``end_epoch``, ``networks``,
``get_snapshot`` / ``restore_from_snapshot``, ``q`` / ``q_target`` /
``target_policy`` / ``qfs`` / ``tfs``.
"""
from collections import OrderedDict

import numpy as np
import torch
from scipy.stats import norm

from . import _lib
from .tp_trainer import _TargetPolicyTrainer


class GaussianTrainer(_TargetPolicyTrainer):
    _kind = _lib.OAC_KIND_GAUSS
    _q_out = 2
    _positive = [False, True]

    def __init__(self, policy_producer, q_producer, n_estimators=2, action_space=None,
                 discount=0.99, reward_scale=1.0, delta=0.95, policy_lr=1e-3, qf_lr=3e-4,
                 std_lr=3e-5, optimizer_class=None, soft_target_tau=1e-2, target_update_period=1,
                 use_automatic_entropy_tuning=False, target_entropy=None, deterministic=True,
                 q_min=0, q_max=100, pac=False, ensemble=False, n_policies=1, share_layers=False,
                 r_mellow_max=1., b_mellow_max=None, mellow_max=False, counts=False,
                 mean_update=False, global_opt=False, std_soft_update=False,
                 std_soft_update_prob=0., train_bias=True, use_target_policy=False,
                 rescale_targets_around_mean=False,
                 device=None, seed=0, use_graph=False, gemm_cfg=-1):
        unsupported = dict(share_layers=not share_layers, deterministic=not deterministic,
                           ensemble=ensemble, global_opt=global_opt)
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(
                "oac_amd.GaussianTrainer implements the g-oac recipe configuration "
                "(share_layers=True, deterministic policy, counts / std_soft_update / "
                f"mean_update / use_target_policy, no ensemble / global-opt); unsupported: {bad}")
        assert not counts or not std_soft_update   # gaussian_trainer.py:88
        self._common_init(device, soft_target_tau, target_update_period, deterministic,
                          discount, reward_scale, policy_lr, qf_lr, use_graph, seed, gemm_cfg)
        self.train_bias = train_bias
        self.std_lr = std_lr
        # gaussian_trainer.py:65-86
        self.action_space = action_space
        self.q_min, self.q_max, self.delta = q_min, q_max, delta
        self.standard_bound = float(norm.ppf(delta, loc=0, scale=1))
        self.share_layers = share_layers
        mean = (q_max + q_min) / 2
        std = (q_max - q_min) / np.sqrt(12)
        self.std_init = std
        self.n_estimators = n_estimators
        self.r_mellow_max, self.b, self.mellow_max = r_mellow_max, b_mellow_max, mellow_max
        self.counts, self.mean_update, self.global_opt = counts, mean_update, global_opt
        self.std_soft_update, self.std_soft_update_prob = std_soft_update, std_soft_update_prob
        self.rescale_targets_around_mean = rescale_targets_around_mean
        self.ensemble, self.n_policies = ensemble, n_policies
        self.use_target_policy = use_target_policy

        # producer call order of the reference constructor: SACTrainer's policy
        # and four critics (unused), the shared-layer critic and its target,
        # then target_policy (gaussian_trainer.py:51-63, 91-99, 146)
        ref_pol = policy_producer()
        for _ in range(4):
            q_producer()
        qb = np.array([mean, np.log(std)])
        ref_q = q_producer(bias=qb, positive=[False, True], train_bias=train_bias)
        ref_qt = q_producer(bias=qb, positive=[False, True], train_bias=train_bias)
        ref_tp = policy_producer()
        self._build(ref_pol, ref_q, ref_qt, ref_tp, policy_lr, qf_lr)
        self._make_target_policy_network(policy_producer)
        self.q, self.q_target = self.qfs[0], self.tfs[0]
        self.q_optimizer = self.qf_optimizers[0]

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.std_bound = self.standard_bound
        c.std_init = float(self.std_init)
        return c

    # ------------------------------------------------------------ diagnostics
    def _fill_eval_statistics(self, plan):
        """gaussian_trainer.py:395-435 (keys and order; 'Policy Loss' is
        mean(upper bound) and 'Policy mu' / 'Policy log std' describe the
        target policy, as in the reference)."""
        v = {k: t.detach().to("cpu").numpy() for k, t in plan.views.items()
             if k in ("q1", "y", "sqe1", "qnew", "head3")}
        Da = self.act_dim
        q_preds = v["q1"][:, :1]
        std_preds = np.exp(v["q1"][:, 1:2])
        st = OrderedDict()
        st["QF mean"] = np.mean(q_preds)
        st["QF std"] = np.mean(std_preds)
        st["QF Loss"] = np.float32(np.mean(v["sqe1"][:, 0]))
        self._stats(st, "Q Predictions", q_preds)
        self._stats(st, "Q Target", v["y"][:, :1])
        st["STD Loss"] = np.float32(np.mean(v["sqe1"][:, 1]))
        self._stats(st, "Q STD Predictions", std_preds)
        self._stats(st, "Q STD Target", v["y"][:, 1:2])
        st["Policy Loss"] = np.mean(v["qnew"])
        self._stats(st, "Policy mu", v["head3"][:, :Da])
        self._stats(st, "Policy log std", np.clip(v["head3"][:, Da:], -20, 2))
        self.eval_statistics = st

    # ------------------------------------------------------------ misc API
    def _qs(self, obs, action):
        with torch.no_grad():
            out = self.q(self._tensor(obs), self._tensor(action))
        return out[:, 0].unsqueeze(-1), out[:, 1].unsqueeze(-1)

    def predict(self, obs, action, std=True):
        """gaussian_trainer.py:161-175."""
        qs, stds = self._qs(obs, action)
        upper_bound = qs + self.standard_bound * stds
        if std:
            return [qs, stds], upper_bound
        return upper_bound

    def obj_func(self, states, actions, upper_bound=False):
        """gaussian_trainer.py:519-529."""
        qs, stds = self._qs(states, actions)
        return qs + self.standard_bound * stds if upper_bound else qs
