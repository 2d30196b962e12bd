"""Drop-in ``ParticleTrainer`` of /root/reference/trainer/particle_trainer_oac.py
(13-449; imported by main.py as ``ParticleTrainerOAC``): the OAC-flavoured
particle trainer (stochastic policy, entropy-tuned SAC policy loss on the
min head), BASELINE configs[4], for the shared-layer K-head critic
(``share_layers``).  main.py selects it for ``--alg p-oac --beta_UB > 0``
(main.py:198-201), though its constructor rejects the kwargs main.py passes
(SURVEY 8a quirk Q3), so callers construct it directly.  The p-oac recipes
themselves run ``oac_amd.ParticleTrainer`` (particle_trainer.py).  The step
runs in liboac_amd (csrc/particle_plan.hip); the interface is the
reference's: constructor kwargs, ``train`` / ``train_from_torch``,
``predict``, ``get_diagnostics``, ``end_epoch``, ``networks``,
``get_snapshot`` / ``restore_from_snapshot``, ``qfs`` / ``tfs`` /
``qf_optimizers``.
"""
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .networks import ArenaFlattenMlp, ArenaTanhGaussianPolicy
from .trainer import AdamStateView, _ArenaTrainer, _dims_from_state, _twin_views, _plain_stats


class ParticleTrainer(_ArenaTrainer):
    _kind = _lib.OAC_KIND_PARTICLE

    def __init__(self, policy_producer, q_producer, n_estimators=2, action_space=None,
                 discount=0.99, reward_scale=1.0, delta=0.95, policy_lr=1e-3, qf_lr=1e-3,
                 optimizer_class=None, soft_target_tau=1e-2, target_update_period=1,
                 use_automatic_entropy_tuning=True, target_entropy=None, deterministic=True,
                 q_min=0, q_max=100, ensemble=False, n_policies=1, share_layers=False,
                 r_mellow_max=1., b_mellow_max=None, mellow_max=False, counts=False,
                 mean_update=False, global_opt=False, std_soft_update=False,
                 std_soft_update_prob=0., train_bias=True, lb=0.1,
                 device=None, seed=0, use_graph=False, gemm_cfg=-1):
        unsupported = dict(share_layers=not share_layers, deterministic=deterministic,
                           ensemble=ensemble, mellow_max=mellow_max,
                           global_opt=global_opt, std_soft_update=std_soft_update)
        bad = [k for k, v in unsupported.items() if v]
        if bad:
            raise NotImplementedError(
                "oac_amd.ParticleTrainerOAC implements the P-OAC configuration "
                "(share_layers=True, stochastic policy, counts, no mellow-max / global-opt / "
                f"std-soft-update); unsupported: {bad}")
        assert not counts or not std_soft_update   # particle_trainer_oac.py:97
        self.train_bias = train_bias
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.use_automatic_entropy_tuning = use_automatic_entropy_tuning
        if use_automatic_entropy_tuning:
            self.target_entropy = target_entropy if target_entropy else \
                -np.prod(action_space.shape).item()
        else:
            self.target_entropy = 0.0
        self.soft_target_tau, self.target_update_period = soft_target_tau, target_update_period
        self.deterministic, self.discount, self.reward_scale = deterministic, discount, reward_scale
        self.policy_lr, self.qf_lr = policy_lr, qf_lr
        self.use_graph, self.seed, self._gemm_cfg = use_graph, int(seed), gemm_cfg
        # quantile bookkeeping, particle_trainer_oac.py:60-74 (delta_index uses p)
        quantiles = [i * 1. / (n_estimators - 1) for i in range(n_estimators)]
        self.delta_index = self.lb_index = None
        for p in range(n_estimators):
            if quantiles[p] >= delta:
                self.delta_index = p
                break
        for p in range(n_estimators):
            if quantiles[p] >= lb:
                self.lb_index = p
                break
        self.share_layers = True
        self.num_particles = n_estimators
        self.n_estimators = 1
        self.q_min, self.q_max, self.delta = q_min, q_max, delta
        self.counts = counts
        self.mean_update = mean_update
        self.global_opt = global_opt
        self.action_space = action_space
        self._q_out = n_estimators

        # producer call order of the reference constructor: SACTrainer's policy +
        # four critics (unused), then the shared-layer critic and its target
        ref_pol = policy_producer()
        for _ in range(4):
            q_producer()
        init_values = np.linspace(q_min, q_max, n_estimators)
        ref_qf = q_producer(bias=init_values, train_bias=train_bias)
        ref_tf = q_producer(bias=init_values, train_bias=train_bias)
        pol_sd = {k: v.detach() for k, v in ref_pol.state_dict().items()}
        Do, Da, H, K = _dims_from_state(pol_sd, ref_qf.state_dict())
        if K != n_estimators:
            raise ValueError("q_producer must build a critic with n_estimators outputs")
        lay = self._alloc(Do, Da, H, self.device)
        self.policy = ArenaTanhGaussianPolicy(self.params, 0, lay, Do, Da, H)
        qf = ArenaFlattenMlp(self.params, lay.q1_base, lay, Do, Da, H, K)
        tf = ArenaFlattenMlp(self.targets, 0, lay, Do, Da, H, K)
        self.policy.load_state_dict(pol_sd)
        qf.load_state_dict({k: v.detach() for k, v in ref_qf.state_dict().items()})
        tf.load_state_dict({k: v.detach() for k, v in ref_tf.state_dict().items()})
        self.policy.oac_trainer = self
        self.qfs, self.tfs = [qf], [tf]
        tw = lambda other, mod: _twin_views(self.params, other, list(mod.parameters()))
        self.policy_optimizer = AdamStateView(self, list(self.policy.parameters()),
                                              tw(self.adam_m, self.policy),
                                              tw(self.adam_v, self.policy), policy_lr,
                                              (0.9, 0.999), 1e-8)
        # train_bias=False: the frozen critic bias has no optimizer state
        q_no_grad = [] if train_bias else \
            [i for i, (n, _) in enumerate(qf.named_parameters()) if n == "last_fc.bias"]
        self.qf_optimizers = [AdamStateView(self, list(qf.parameters()), tw(self.adam_m, qf),
                                            tw(self.adam_v, qf), qf_lr, (0.9, 0.999), 1e-8,
                                            no_grad=q_no_grad)]
        self.alpha_optimizer = AdamStateView(self, [self.log_alpha], [self.alpha_state[1:2]],
                                             [self.alpha_state[2:3]], policy_lr, (0.9, 0.999),
                                             1e-8)
        self.eval_statistics = OrderedDict()
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.freeze_q_bias = int(not self.train_bias)
        return c

    # ------------------------------------------------------------ diagnostics
    def _fill_eval_statistics(self, plan):
        """particle_trainer_oac.py:329-362 (keys and order)."""
        v = {k: t.detach().to("cpu").numpy() for k, t in plan.views.items()
             if k in ("q1", "tq1", "sqe1", "logp1", "head1", "qnew")}
        K, Da = self.num_particles, self.act_dim
        qs, tq = v["q1"], v["tq1"]
        sorted_qs = np.sort(qs, axis=1).T[:, :, None]          # [K, B, 1]
        order = np.arange(K)[None, :]
        st = OrderedDict()
        st["QF mean"] = np.mean(sorted_qs, axis=0).mean()
        st["QF std"] = np.std(sorted_qs, axis=0).mean()
        st["QF Unordered"] = np.float64(np.sum(np.argsort(qs, axis=1, kind="stable") != order))
        st["QF target Undordered"] = np.float64(
            np.sum(np.argsort(tq, axis=1, kind="stable") != order))
        for i in range(K):
            st[f"QF{i} Loss"] = np.float32(np.mean(v["sqe1"][:, i]))
            for name, arr in ((f"Q{i}Predictions", sorted_qs[i]), (f"Q{i}Targets", tq[:, i:i + 1])):
                st[name + " Mean"] = np.mean(arr)
                st[name + " Std"] = np.std(arr)
                st[name + " Max"] = np.max(arr)
                st[name + " Min"] = np.min(arr)
        alpha = float(self.alpha_state[3].item()) if self.use_automatic_entropy_tuning else 0.0
        st["Policy Loss"] = np.mean(alpha * v["logp1"][:, 0] - v["qnew"][:, 0])
        mean = v["head1"][:, :Da]
        log_std = np.clip(v["head1"][:, Da:], -20, 2)
        for name, arr in (("Policy mu", mean), ("Policy log std", log_std)):
            st[name + " Mean"] = np.mean(arr)
            st[name + " Std"] = np.std(arr)
            st[name + " Max"] = np.max(arr)
            st[name + " Min"] = np.min(arr)
        self.eval_statistics = st

    def get_diagnostics(self):
        return self.eval_statistics

    def end_epoch(self, epoch):
        self._need_to_update_eval_statistics = True

    def predict(self, obs, action, all_particles=False, upper_bound=True, beta_UB=None):
        """particle_trainer_oac.py:147-167 (share_layers: the K heads of the one
        critic are the particles), on oac_critic_eval; differentiable w.r.t.
        obs and action like the reference's."""
        from .networks import critics_apply
        q = critics_apply([self.qfs[0]], obs, action)
        if q.dim() == 1:
            q = q.unsqueeze(0)
        qs = q.t().unsqueeze(-1)                  # [K, B, 1] (stack + permute(2, 1, 0))
        if upper_bound:
            if self.delta_index is None:
                raise ValueError("predict(upper_bound=True) needs delta_index: delta must be a "
                                 "quantile level in (0, 1) (particle_trainer_oac.py:60-67), "
                                 f"got delta={self.delta}")
            out = torch.sort(qs, dim=0)[0][self.delta_index]
        else:
            out = torch.mean(qs, dim=0)
        if all_particles:
            return torch.sort(qs, dim=0)[0], out
        return out

    @property
    def networks(self):
        return [self.policy] + self.qfs + self.tfs

    def get_snapshot(self):
        data = dict(policy_state_dict=self.policy.state_dict(),
                    policy_optim_state_dict=self.policy_optimizer.state_dict(),
                    eval_statistics=_plain_stats(self.eval_statistics),
                    _n_train_steps_total=self._n_train_steps_total,
                    _need_to_update_eval_statistics=self._need_to_update_eval_statistics)
        if self.use_automatic_entropy_tuning:
            data["alpha_optim_state_dict"] = self.alpha_optimizer.state_dict()
            data["log_alpha"] = self.log_alpha
        data["qfs_state_dicts"] = [q.state_dict() for q in self.qfs]
        data["qfs_optims_state_dicts"] = [o.state_dict() for o in self.qf_optimizers]
        data["target_qfs_state_dicts"] = [t.state_dict() for t in self.tfs]
        return data

    def restore_from_snapshot(self, ss):
        self.policy.load_state_dict(ss["policy_state_dict"])
        self.policy_optimizer.load_state_dict(ss["policy_optim_state_dict"])
        for i in range(len(ss["qfs_state_dicts"])):
            self.qfs[i].load_state_dict(ss["qfs_state_dicts"][i])
            self.qf_optimizers[i].load_state_dict(ss["qfs_optims_state_dicts"][i])
            self.tfs[i].load_state_dict(ss["target_qfs_state_dicts"][i])
        if self.use_automatic_entropy_tuning:
            self.log_alpha.copy_(torch.as_tensor(ss["log_alpha"]).reshape(1))
            self.alpha_optimizer.load_state_dict(ss["alpha_optim_state_dict"])
            self.alpha_state[3] = torch.exp(self.log_alpha[0])
        self.eval_statistics = ss["eval_statistics"]
        self._n_train_steps_total = int(ss["_n_train_steps_total"])
        self._need_to_update_eval_statistics = ss["_need_to_update_eval_statistics"]
        self.step_state[0] = self._n_train_steps_total
