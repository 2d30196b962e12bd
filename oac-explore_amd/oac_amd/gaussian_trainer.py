"""Drop-in ``GaussianTrainer`` of the g-oac recipes
(/root/reference/trainer/gaussian_trainer.py:14-538, the trainer main.py
builds for ``--alg g-oac``, main.py:219-233), in the configuration every
reproduce_g-oac*.sh recipe runs: ``--share_layers`` (one critic with two
outputs, Q mean | log std, exp'd by ``positive=[False, True]``), the
deterministic policy (GaussianTrainer's default, not overridden for g-oac),
optionally ``--counts`` / ``std_soft_update``.  The step runs in liboac_amd
(csrc/gauss_plan.hip); the interface is the reference's: constructor kwargs,
``train`` / ``train_from_torch``, ``predict``, ``obj_func``,
``get_diagnostics``, ``end_epoch``, ``networks``, ``get_snapshot`` /
``restore_from_snapshot``, ``q`` / ``q_target`` / ``target_policy`` /
``qfs`` / ``tfs``.
"""
from collections import OrderedDict

import numpy as np
import torch
from scipy.stats import norm

from . import _lib
from .networks import ArenaFlattenMlp, ArenaTanhGaussianPolicy
from .trainer import AdamStateView, _ArenaTrainer, _dims_from_state, _twin_views, _plain_stats

_LOG_STD_HEAD = ("last_fc_log_std.weight", "last_fc_log_std.bias")


class GaussianTrainer(_ArenaTrainer):
    _kind = _lib.OAC_KIND_GAUSS
    _q_out = 2

    def __init__(self, policy_producer, q_producer, n_estimators=2, action_space=None,
                 discount=0.99, reward_scale=1.0, delta=0.95, policy_lr=1e-3, qf_lr=3e-4,
                 std_lr=3e-5, optimizer_class=None, soft_target_tau=1e-2, target_update_period=1,
                 use_automatic_entropy_tuning=False, target_entropy=None, deterministic=True,
                 q_min=0, q_max=100, pac=False, ensemble=False, n_policies=1, share_layers=False,
                 r_mellow_max=1., b_mellow_max=None, mellow_max=False, counts=False,
                 mean_update=False, global_opt=False, std_soft_update=False,
                 std_soft_update_prob=0., train_bias=True, use_target_policy=False,
                 rescale_targets_around_mean=False,
                 device=None, seed=0, use_graph=True, gemm_cfg=-1):
        unsupported = dict(share_layers=not share_layers, deterministic=not deterministic,
                           ensemble=ensemble, global_opt=global_opt, mean_update=mean_update,
                           use_target_policy=use_target_policy, train_bias=not train_bias)
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(
                "oac_amd.GaussianTrainer implements the g-oac recipe configuration "
                "(share_layers=True, deterministic policy, counts / std_soft_update, "
                f"trainable bias, no ensemble / global-opt / mean-update); unsupported: {bad}")
        assert not counts or not std_soft_update   # gaussian_trainer.py:88
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        # SACTrainer.__init__ bookkeeping (the entropy term is unused by this step)
        self.use_automatic_entropy_tuning = False
        self.target_entropy = 0.0
        self.soft_target_tau, self.target_update_period = soft_target_tau, target_update_period
        self.deterministic, self.discount, self.reward_scale = deterministic, discount, reward_scale
        self.policy_lr, self.qf_lr, self.std_lr = policy_lr, qf_lr, std_lr
        self.use_graph, self.seed, self._gemm_cfg = use_graph, int(seed), gemm_cfg
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
        pol_sd = {k: v.detach() for k, v in ref_pol.state_dict().items()}
        Do, Da, H, K = _dims_from_state(pol_sd, ref_q.state_dict())
        if K != 2:
            raise ValueError("share_layers: q_producer must build a critic with 2 outputs")
        lay = self._alloc(Do, Da, H, self.device)
        self.policy = ArenaTanhGaussianPolicy(self.params, 0, lay, Do, Da, H)
        self.target_policy = ArenaTanhGaussianPolicy(self.params, lay.tpol_base, lay, Do, Da, H)
        self.q = ArenaFlattenMlp(self.params, lay.q1_base, lay, Do, Da, H, 2,
                                 positive=[False, True])
        self.q_target = ArenaFlattenMlp(self.targets, 0, lay, Do, Da, H, 2, positive=[False, True])
        self.policy.load_state_dict(pol_sd)
        self.target_policy.load_state_dict({k: v.detach() for k, v in ref_tp.state_dict().items()})
        self.q.load_state_dict({k: v.detach() for k, v in ref_q.state_dict().items()})
        self.q_target.load_state_dict({k: v.detach() for k, v in ref_qt.state_dict().items()})
        self.policy.oac_trainer = self
        self.qfs, self.tfs = [self.q], [self.q_target]
        tw = lambda other, mod: _twin_views(self.params, other, list(mod.parameters()))
        names = [n for n, _ in self.policy.named_parameters()]
        no_grad = [i for i, n in enumerate(names) if n in _LOG_STD_HEAD]   # deterministic policy

        def popt(mod):
            return AdamStateView(self, list(mod.parameters()), tw(self.adam_m, mod),
                                 tw(self.adam_v, mod), policy_lr, (0.9, 0.999), 1e-8,
                                 no_grad=no_grad)
        self.policy_optimizer = popt(self.policy)
        self.target_policy_optimizer = popt(self.target_policy)
        self.q_optimizer = AdamStateView(self, list(self.q.parameters()), tw(self.adam_m, self.q),
                                         tw(self.adam_v, self.q), qf_lr, (0.9, 0.999), 1e-8)
        self.qf_optimizers = [self.q_optimizer]
        # SACTrainer's alpha (snapshot keys only; g-oac does not tune it)
        self.alpha_optimizer = AdamStateView(self, [self.log_alpha], [self.alpha_state[1:2]],
                                             [self.alpha_state[2:3]], policy_lr, (0.9, 0.999),
                                             1e-8)
        self.eval_statistics = OrderedDict()
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.std_bound = self.standard_bound
        c.std_init = float(self.std_init)
        c.std_soft_prob = float(self.std_soft_update_prob) if self.std_soft_update else -1.0
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

        def stats(name, arr):
            st[name + " Mean"] = np.mean(arr)
            st[name + " Std"] = np.std(arr)
            st[name + " Max"] = np.max(arr)
            st[name + " Min"] = np.min(arr)
        st["QF mean"] = np.mean(q_preds)
        st["QF std"] = np.mean(std_preds)
        st["QF Loss"] = np.float32(np.mean(v["sqe1"][:, 0]))
        stats("Q Predictions", q_preds)
        stats("Q Target", v["y"][:, :1])
        st["STD Loss"] = np.float32(np.mean(v["sqe1"][:, 1]))
        stats("Q STD Predictions", std_preds)
        stats("Q STD Target", v["y"][:, 1:2])
        st["Policy Loss"] = np.mean(v["qnew"])
        stats("Policy mu", v["head3"][:, :Da])
        stats("Policy log std", np.clip(v["head3"][:, Da:], -20, 2))
        self.eval_statistics = st

    def get_diagnostics(self):
        return self.eval_statistics

    def end_epoch(self, epoch):
        self._need_to_update_eval_statistics = True

    # ------------------------------------------------------------ misc API
    def _qs(self, obs, action):
        obs = torch.as_tensor(np.asarray(obs) if not torch.is_tensor(obs) else obs,
                              dtype=torch.float32, device=self.device)
        action = torch.as_tensor(np.asarray(action) if not torch.is_tensor(action) else action,
                                 dtype=torch.float32, device=self.device)
        with torch.no_grad():
            out = self.q(obs, action)
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

    @property
    def networks(self):
        return [self.policy] + self.qfs + self.tfs + [self.target_policy]

    def get_snapshot(self):
        """gaussian_trainer.py:452-482 (keys)."""
        return dict(policy_state_dict=self.policy.state_dict(),
                    policy_optim_state_dict=self.policy_optimizer.state_dict(),
                    log_alpha=self.log_alpha,
                    alpha_optim_state_dict=self.alpha_optimizer.state_dict(),
                    eval_statistics=_plain_stats(self.eval_statistics),
                    _n_train_steps_total=self._n_train_steps_total,
                    _need_to_update_eval_statistics=self._need_to_update_eval_statistics,
                    qfs_state_dicts=[self.q.state_dict()],
                    qfs_optims_state_dicts=[self.q_optimizer.state_dict()],
                    target_qfs_state_dicts=[self.q_target.state_dict()],
                    target_policy_state_dict=self.target_policy.state_dict(),
                    target_policy_opt_state_dict=self.target_policy_optimizer.state_dict())

    def restore_from_snapshot(self, ss):
        """gaussian_trainer.py:484-517."""
        self.policy.load_state_dict(ss["policy_state_dict"])
        self.policy_optimizer.load_state_dict(ss["policy_optim_state_dict"])
        self.q.load_state_dict(ss["qfs_state_dicts"][0])
        self.q_optimizer.load_state_dict(ss["qfs_optims_state_dicts"][0])
        self.q_target.load_state_dict(ss["target_qfs_state_dicts"][0])
        self.log_alpha.copy_(torch.as_tensor(ss["log_alpha"]).reshape(1))
        self.alpha_optimizer.load_state_dict(ss["alpha_optim_state_dict"])
        self.eval_statistics = ss["eval_statistics"]
        self._n_train_steps_total = int(ss["_n_train_steps_total"])
        self._need_to_update_eval_statistics = ss["_need_to_update_eval_statistics"]
        self.target_policy.load_state_dict(ss["target_policy_state_dict"])
        self.target_policy_optimizer.load_state_dict(ss["target_policy_opt_state_dict"])
        self.step_state[0] = self._n_train_steps_total
