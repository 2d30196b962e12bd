"""Drop-in ``ParticleTrainer`` of /root/reference/trainer/particle_trainer.py
(12-525): the trainer main.py builds for ``--alg p-oac`` without
``--beta_UB`` (main.py:198-204, 364, 488-490) -- i.e. every reproduce_p-oac*.sh
recipe -- with the shared-layer K-particle critic (``--share_layers``), the
deterministic policy (``deterministic = not --stochastic``), and optionally
``--counts`` / ``std_soft_update`` / ``--mean_update`` /
``rescale_targets_around_mean``.  Per step: sorted-particle TD targets with
the critic loss averaged over particles, the policy maximising the
``delta_index``-th sorted particle of the post-step critic, the target policy
its particle mean, Polyak.  The step runs in liboac_amd (csrc/det_plan.hip);
the interface is the reference's: constructor kwargs, ``train`` /
``train_from_torch``, ``predict``, ``obj_func``, ``get_diagnostics``,
``end_epoch``, ``networks``, ``get_snapshot`` / ``restore_from_snapshot``,
``qfs`` / ``tfs`` / ``qf_optimizers`` / ``target_policy``.
"""
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .tp_trainer import _TargetPolicyTrainer


class ParticleTrainer(_TargetPolicyTrainer):
    _kind = _lib.OAC_KIND_PARTICLE_UB

    def __init__(self, policy_producer, q_producer, n_estimators=2, action_space=None,
                 discount=0.99, reward_scale=1.0, delta=0.95, policy_lr=1e-3, qf_lr=1e-3,
                 optimizer_class=None, soft_target_tau=1e-2, target_update_period=1,
                 use_automatic_entropy_tuning=False, target_entropy=None, deterministic=True,
                 q_min=0, q_max=100, ensemble=False, n_policies=1, share_layers=False,
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
                "oac_amd.ParticleTrainer implements the p-oac recipe configuration "
                "(share_layers=True, deterministic policy, counts / std_soft_update / "
                "mean_update / rescale_targets_around_mean / train_bias / "
                f"use_target_policy, no ensemble / global-opt); unsupported: {bad}")
        assert not counts or not std_soft_update   # particle_trainer.py:92
        self._common_init(device, soft_target_tau, target_update_period, deterministic,
                          discount, reward_scale, policy_lr, qf_lr, use_graph, seed, gemm_cfg)
        self.train_bias = train_bias
        # quantile bookkeeping, particle_trainer.py:61-69 (delta_index uses p - 1
        # when the quantile grid steps over delta)
        quantiles = [i * 1. / (n_estimators - 1) for i in range(n_estimators)]
        for p in range(n_estimators):
            if quantiles[p] == delta:
                self.delta_index = p
                break
            if quantiles[p] > delta:
                self.delta_index = p - 1
                break
        self.share_layers = share_layers
        self.num_particles = n_estimators
        self.n_estimators = 1
        self._q_out = n_estimators
        self.q_min, self.q_max, self.delta = q_min, q_max, delta
        self.r_mellow_max, self.b, self.mellow_max = r_mellow_max, b_mellow_max, mellow_max
        self.counts, self.mean_update, self.global_opt = counts, mean_update, global_opt
        self.std_soft_update, self.std_soft_update_prob = std_soft_update, std_soft_update_prob
        self.rescale_targets_around_mean = rescale_targets_around_mean
        self.action_space = action_space
        self.ensemble, self.n_policies = ensemble, n_policies
        self.use_target_policy = use_target_policy

        # producer call order of the reference constructor: SACTrainer's policy
        # and four critics (unused), the shared-layer critic and its target
        # (the target then copied from the critic, soft_update tau=1), then
        # target_policy (particle_trainer.py:47-59, 96-106, 141)
        ref_pol = policy_producer()
        for _ in range(4):
            q_producer()
        init_values = np.linspace(q_min, q_max, n_estimators)
        ref_q = q_producer(bias=init_values, train_bias=train_bias)
        q_producer(bias=init_values, train_bias=train_bias)
        ref_tp = policy_producer()
        self._build(ref_pol, ref_q, ref_q, ref_tp, policy_lr, qf_lr)
        self._make_target_policy_network(policy_producer)

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.delta_index = int(self.delta_index)
        c.rescale_spread = float(self.q_max - self.q_min) if self.rescale_targets_around_mean \
            else 0.0
        return c

    # ------------------------------------------------------------ diagnostics
    def _fill_eval_statistics(self, plan):
        """particle_trainer.py:362-403 (keys and order; 'Policy Loss' is
        mean(upper bound) and 'Policy mu' / 'Policy log std' describe the
        target policy, as in the reference)."""
        v = {k: t.detach().to("cpu").numpy() for k, t in plan.views.items()
             if k in ("q1", "tq1", "sqe1", "qnew", "head3")}
        K, Da = self.num_particles, self.act_dim
        qs, tq = v["q1"], v["tq1"]
        sorted_qs = np.sort(qs, axis=1).T[:, :, None]          # [K, B, 1]
        order = np.arange(K)[None, :]
        losses = [np.float32(np.mean(v["sqe1"][:, i])) for i in range(K)]
        st = OrderedDict()
        st["QF mean"] = np.mean(sorted_qs, axis=0).mean()
        st["QF std"] = np.std(sorted_qs, axis=0).mean()
        st["QF Unordered"] = np.float64(np.sum(np.argsort(qs, axis=1, kind="stable") != order))
        st["QF target Undordered"] = np.float64(
            np.sum(np.argsort(tq, axis=1, kind="stable") != order))
        st["Q Loss"] = np.float32(np.sum(losses, dtype=np.float32) / np.float32(K))
        for i in range(K):
            st[f"QF{i} Loss"] = losses[i]
            self._stats(st, f"Q{i}Predictions", sorted_qs[i])
            self._stats(st, f"Q{i}Targets", tq[:, i:i + 1])
        st["Policy Loss"] = np.mean(v["qnew"])
        self._stats(st, "Policy mu", v["head3"][:, :Da])
        self._stats(st, "Policy log std", np.clip(v["head3"][:, Da:], -20, 2))
        self.eval_statistics = st

    # ------------------------------------------------------------ misc API
    def _sorted(self, obs, action):
        with torch.no_grad():
            qs = self.qfs[0](self._tensor(obs), self._tensor(action)).t().unsqueeze(-1)
        return qs, torch.sort(qs, dim=0)[0]                     # [K, B, 1]

    def predict(self, obs, action, all_particles=False):
        """particle_trainer.py:160-174."""
        _, sorted_qs = self._sorted(obs, action)
        upper_bound = sorted_qs[self.delta_index]
        if all_particles:
            return sorted_qs, upper_bound
        return upper_bound

    def obj_func(self, states, actions, upper_bound=False):
        """particle_trainer.py:507-518."""
        qs, sorted_qs = self._sorted(states, actions)
        return sorted_qs[self.delta_index] if upper_bound else torch.mean(qs, dim=0)
