"""Shared host side of the deterministic-policy trainers with a separately
trained ``target_policy`` -- g-oac ``GaussianTrainer``
(/root/reference/trainer/gaussian_trainer.py) and the p-oac
``ParticleTrainer`` (/root/reference/trainer/particle_trainer.py).  Both are
``SACTrainer`` subclasses in the reference with the same network set
(policy, one shared-layer critic and its target, target_policy), the same
optimizer set and the same snapshot keys; their steps run in liboac_amd
(csrc/det_plan.hip) over the arena [policy | target_policy | critic].
"""
from collections import OrderedDict

import numpy as np
import torch

from .networks import ArenaFlattenMlp, ArenaTanhGaussianPolicy
from .trainer import AdamStateView, _ArenaTrainer, _dims_from_state, _twin_views, _plain_stats

_LOG_STD_HEAD = ("last_fc_log_std.weight", "last_fc_log_std.bias")


class _TargetPolicyTrainer(_ArenaTrainer):
    _positive = False       # critic output exp (FlattenMlp positive=..., networks.py:69-75)

    def _common_init(self, device, soft_target_tau, target_update_period, deterministic,
                     discount, reward_scale, policy_lr, qf_lr, use_graph, seed, gemm_cfg):
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        # SACTrainer.__init__ bookkeeping (no entropy term in these steps)
        self.use_automatic_entropy_tuning = False
        self.target_entropy = 0.0
        self.soft_target_tau, self.target_update_period = soft_target_tau, target_update_period
        self.deterministic, self.discount, self.reward_scale = deterministic, discount, reward_scale
        self.policy_lr, self.qf_lr = policy_lr, qf_lr
        self.use_graph, self.seed, self._gemm_cfg = use_graph, int(seed), gemm_cfg

    def _build(self, ref_pol, ref_q, ref_qt, ref_tp, policy_lr, qf_lr):
        """Arena modules initialised from the producers' state_dicts, and the
        reference's optimizer views (policy, target_policy, shared critic)."""
        pol_sd = {k: v.detach() for k, v in ref_pol.state_dict().items()}
        Do, Da, H, K = _dims_from_state(pol_sd, ref_q.state_dict())
        if K != self._q_out:
            raise ValueError(f"share_layers: q_producer must build a critic with {self._q_out} "
                             f"outputs, got {K}")
        lay = self._alloc(Do, Da, H, self.device)
        self.policy = ArenaTanhGaussianPolicy(self.params, 0, lay, Do, Da, H)
        self.target_policy = ArenaTanhGaussianPolicy(self.params, lay.tpol_base, lay, Do, Da, H)
        qf = ArenaFlattenMlp(self.params, lay.q1_base, lay, Do, Da, H, K, positive=self._positive)
        tf = ArenaFlattenMlp(self.targets, 0, lay, Do, Da, H, K, positive=self._positive)
        self.policy.load_state_dict(pol_sd)
        self.target_policy.load_state_dict({k: v.detach() for k, v in ref_tp.state_dict().items()})
        qf.load_state_dict({k: v.detach() for k, v in ref_q.state_dict().items()})
        tf.load_state_dict({k: v.detach() for k, v in ref_qt.state_dict().items()})
        self.policy.oac_trainer = self
        self.qfs, self.tfs = [qf], [tf]
        tw = lambda other, mod: _twin_views(self.params, other, list(mod.parameters()))
        names = [n for n, _ in self.policy.named_parameters()]
        # deterministic policies: the log-std heads never get a gradient
        no_grad = [i for i, n in enumerate(names) if n in _LOG_STD_HEAD]

        def popt(mod):
            return AdamStateView(self, list(mod.parameters()), tw(self.adam_m, mod),
                                 tw(self.adam_v, mod), policy_lr, (0.9, 0.999), 1e-8,
                                 no_grad=no_grad)
        self.policy_optimizer = popt(self.policy)
        self.target_policy_optimizer = popt(self.target_policy)
        q_no_grad = [] if self.train_bias else \
            [i for i, (n, _) in enumerate(qf.named_parameters()) if n == "last_fc.bias"]
        self.qf_optimizers = [AdamStateView(self, list(qf.parameters()), tw(self.adam_m, qf),
                                            tw(self.adam_v, qf), qf_lr, (0.9, 0.999), 1e-8,
                                            no_grad=q_no_grad)]
        # SACTrainer's alpha (snapshot keys only)
        self.alpha_optimizer = AdamStateView(self, [self.log_alpha], [self.alpha_state[1:2]],
                                             [self.alpha_state[2:3]], policy_lr, (0.9, 0.999),
                                             1e-8)
        self.eval_statistics = OrderedDict()
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True

    def _make_target_policy_network(self, policy_producer):
        """use_target_policy without mean_update (particle_trainer.py:150-154,
        gaussian_trainer.py:154-158): a policy_producer() network overwritten
        with a copy of the policy (soft update, tau 1) that supplies the next
        actions of the TD target (:196-199).  The reference's per-step soft
        update copies this network onto itself (:386-388 / :385-387), so it
        keeps the weights it has -- here a frozen block outside the Adam arena
        (oac_sac_buffers.next_policy), loadable like the reference's."""
        self.target_policy_network = None
        self._tpn = None
        if not (self.use_target_policy and not self.mean_update):
            return
        policy_producer()   # the reference's producer call (its init is overwritten)
        lay = self.layout
        self._tpn = self.params[:lay.pol_size].clone()
        self.target_policy_network = ArenaTanhGaussianPolicy(
            self._tpn, 0, lay, self.obs_dim, self.act_dim, self.hidden)

    def _next_policy_ptr(self):
        return None if getattr(self, "_tpn", None) is None else self._tpn.data_ptr()

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.std_soft_update = int(bool(self.std_soft_update))
        c.std_soft_prob = float(self.std_soft_update_prob)
        c.mean_update = int(bool(self.mean_update))
        c.freeze_q_bias = int(not self.train_bias)
        return c

    @staticmethod
    def _stats(st, name, arr):
        """create_stats_ordered_dict (utils/eval_util.py) for one array."""
        st[name + " Mean"] = np.mean(arr)
        st[name + " Std"] = np.std(arr)
        st[name + " Max"] = np.max(arr)
        st[name + " Min"] = np.min(arr)

    def _tensor(self, x):
        return torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x,
                               dtype=torch.float32, device=self.device)

    def get_diagnostics(self):
        return self.eval_statistics

    def end_epoch(self, epoch):
        self._need_to_update_eval_statistics = True

    @property
    def networks(self):
        nets = [self.policy] + self.qfs + self.tfs + [self.target_policy]
        if getattr(self, "target_policy_network", None) is not None:
            nets.append(self.target_policy_network)
        return nets

    def get_snapshot(self):
        """gaussian_trainer.py:452-482 / particle_trainer.py:449-478 (keys)."""
        d = dict(policy_state_dict=self.policy.state_dict(),
                    policy_optim_state_dict=self.policy_optimizer.state_dict(),
                    log_alpha=self.log_alpha,
                    alpha_optim_state_dict=self.alpha_optimizer.state_dict(),
                    eval_statistics=_plain_stats(self.eval_statistics),
                    _n_train_steps_total=self._n_train_steps_total,
                    _need_to_update_eval_statistics=self._need_to_update_eval_statistics,
                    qfs_state_dicts=[q.state_dict() for q in self.qfs],
                    qfs_optims_state_dicts=[o.state_dict() for o in self.qf_optimizers],
                    target_qfs_state_dicts=[t.state_dict() for t in self.tfs],
                    target_policy_state_dict=self.target_policy.state_dict(),
                    target_policy_opt_state_dict=self.target_policy_optimizer.state_dict())
        if getattr(self, "target_policy_network", None) is not None:
            d["target_policy_network"] = self.target_policy_network.state_dict()
        return d

    def restore_from_snapshot(self, ss):
        """gaussian_trainer.py:484-517 / particle_trainer.py:480-505."""
        self.policy.load_state_dict(ss["policy_state_dict"])
        self.policy_optimizer.load_state_dict(ss["policy_optim_state_dict"])
        for i in range(len(ss["qfs_state_dicts"])):
            self.qfs[i].load_state_dict(ss["qfs_state_dicts"][i])
            self.qf_optimizers[i].load_state_dict(ss["qfs_optims_state_dicts"][i])
            self.tfs[i].load_state_dict(ss["target_qfs_state_dicts"][i])
        self.log_alpha.copy_(torch.as_tensor(ss["log_alpha"]).reshape(1))
        self.alpha_optimizer.load_state_dict(ss["alpha_optim_state_dict"])
        self.eval_statistics = ss["eval_statistics"]
        self._n_train_steps_total = int(ss["_n_train_steps_total"])
        self._need_to_update_eval_statistics = ss["_need_to_update_eval_statistics"]
        self.target_policy.load_state_dict(ss["target_policy_state_dict"])
        self.target_policy_optimizer.load_state_dict(ss["target_policy_opt_state_dict"])
        if getattr(self, "target_policy_network", None) is not None:
            self.target_policy_network.load_state_dict(ss["target_policy_network"])
        self.step_state[0] = self._n_train_steps_total
