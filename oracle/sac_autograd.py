"""CPU restatement of SACTrainer.train_from_torch on torch autograd -- the
reference's own op sequence, for the CPU baseline.

TEST INFRASTRUCTURE ONLY (like sac_oracle.py): nothing in the product may
import it.  ``bench.py``'s ``cpu_baseline`` leg times it on the GPU box's host
cores; tests/test_oracle_golden.py pins it against the reference-run goldens.

Where ``sac_oracle.SACOracle`` writes every backward pass out by hand (the
minimal products), this one runs the reference's forward ops with autograd
and lets ``backward()`` do what the reference's does -- including its wasted
work (critic weight gradients and the full [obs | act] input gradient in the
policy backward), so its timing is the reference's cost on the same host:

* networks   FlattenMlp / Mlp.forward        /root/reference/networks.py:62-79,159-161
             TanhGaussianPolicy.forward       /root/reference/trainer/policies.py:260-316
             TanhNormal.rsample / log_prob    /root/reference/trainer/policies.py:147-160,175-192
* the step   SACTrainer.train_from_torch      /root/reference/trainer/trainer.py:126-224
             (alpha loss and step, min Q on the fresh actions, critic MSE,
             Q1 / Q2 / policy zero_grad-backward-step in that order, Polyak)
* optimiser  torch 1.4 optim.Adam.step, parameters updated through ``.data``
             (trainer/trainer.py:75-91): the version counter does not move,
             so ``policy_loss.backward()`` runs through the post-step critic
             weights with the pre-step activations -- quirk Q1 of SURVEY 8a
* Polyak     soft_update_from_to              /root/reference/utils/pytorch_util.py:5-9

The standard-normal draws behind ``Normal(0, 1).sample()`` are explicit
inputs (eps1 for policy(obs), eps2 for policy(next_obs)), as in sac_oracle.
"""
import math

import torch
from torch import nn

LOG_SIG_MAX = 2.0    # trainer/policies.py:10
LOG_SIG_MIN = -20.0  # trainer/policies.py:11


def _param(x, dtype):
    return nn.Parameter(torch.as_tensor(x).to(dtype).clone())


class _Mlp(nn.Module):
    """Mlp (networks.py:17-79): fc0.., last_fc (+ last_fc_log_std for the policy)."""

    def __init__(self, sd, dtype, policy=False):
        super().__init__()
        n = sum(1 for k in sd if k.startswith("fc") and k.endswith(".weight"))
        self.fcs = nn.ModuleList()
        for i in range(n):
            lin = nn.Linear(1, 1)
            lin.weight = _param(sd[f"fc{i}.weight"], dtype)
            lin.bias = _param(sd[f"fc{i}.bias"], dtype)
            self.fcs.append(lin)
        self.last_fc = nn.Linear(1, 1)
        self.last_fc.weight = _param(sd["last_fc.weight"], dtype)
        self.last_fc.bias = _param(sd["last_fc.bias"], dtype)
        if policy:
            self.last_fc_log_std = nn.Linear(1, 1)
            self.last_fc_log_std.weight = _param(sd["last_fc_log_std.weight"], dtype)
            self.last_fc_log_std.bias = _param(sd["last_fc_log_std.bias"], dtype)

    def trunk(self, h):
        for fc in self.fcs:
            h = torch.relu(fc(h))
        return h

    def q(self, obs, act):   # FlattenMlp.forward: cat then Mlp.forward (identity output)
        return self.last_fc(self.trunk(torch.cat([obs, act], dim=1)))

    def named(self):
        """{reference state_dict key: parameter}"""
        out = {}
        for i, fc in enumerate(self.fcs):
            out[f"fc{i}.weight"], out[f"fc{i}.bias"] = fc.weight, fc.bias
        out["last_fc.weight"], out["last_fc.bias"] = self.last_fc.weight, self.last_fc.bias
        if hasattr(self, "last_fc_log_std"):
            out["last_fc_log_std.weight"] = self.last_fc_log_std.weight
            out["last_fc_log_std.bias"] = self.last_fc_log_std.bias
        return out

    def policy(self, obs, eps):
        """TanhGaussianPolicy.forward(reparameterize=True, return_log_prob=True):
        (action, mean, log_std, log_prob) with TanhNormal's rsample / log_prob."""
        h = self.trunk(obs)
        mean = self.last_fc(h)
        log_std = torch.clamp(self.last_fc_log_std(h), LOG_SIG_MIN, LOG_SIG_MAX)
        std = torch.exp(log_std)
        z = mean + std * eps                                   # policies.py:182-186
        a = torch.tanh(z)
        # Normal(mean, std).log_prob(z) - log(1 - tanh(z)^2 + 1e-6)  (policies.py:154-160)
        lp = -((z - mean) ** 2) / (2 * std ** 2) - std.log() - math.log(math.sqrt(2 * math.pi))
        lp = lp - torch.log(1 - a * a + 1e-6)
        return a, mean, log_std, lp.sum(dim=1, keepdim=True)


class Adam14:
    """torch 1.4.0 optim.Adam.step over parameters' .grad, updates via .data."""

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = [torch.zeros_like(p.data) for p in self.params]
        self.v = [torch.zeros_like(p.data) for p in self.params]
        self.t = 0

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def step(self):
        self.t += 1
        bc1, bc2 = 1 - self.b1 ** self.t, 1 - self.b2 ** self.t
        with torch.no_grad():
            for p, m, v in zip(self.params, self.m, self.v):
                g = p.grad
                m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
                p.data.addcdiv_(m, denom, value=-(self.lr / bc1))


class SACAutograd:
    """SACTrainer (trainer/trainer.py:14-280) on torch autograd, CPU."""

    def __init__(self, params, obs_dim, act_dim, discount=0.99, reward_scale=1.0, policy_lr=3e-4,
                 qf_lr=3e-4, tau=5e-3, target_update_period=1, auto_alpha=True,
                 target_entropy=None, log_alpha0=0.0, dtype=torch.float32):
        self.dtype = dtype
        self.policy = _Mlp(params["policy"], dtype, policy=True)
        self.qf1, self.qf2 = _Mlp(params["qf1"], dtype), _Mlp(params["qf2"], dtype)
        self.target_qf1 = _Mlp(params["target_qf1"], dtype)
        self.target_qf2 = _Mlp(params["target_qf2"], dtype)
        self.discount, self.reward_scale, self.tau = discount, reward_scale, tau
        self.period, self.auto_alpha = target_update_period, auto_alpha
        self.target_entropy = -float(act_dim) if target_entropy is None else target_entropy
        self.log_alpha = torch.full((1,), float(log_alpha0), dtype=dtype, requires_grad=True)
        self.policy_optimizer = Adam14(self.policy.parameters(), policy_lr)
        self.qf1_optimizer = Adam14(self.qf1.parameters(), qf_lr)
        self.qf2_optimizer = Adam14(self.qf2.parameters(), qf_lr)
        self.alpha_optimizer = Adam14([self.log_alpha], policy_lr)
        self.n_steps = 0

    def step(self, batch, eps1, eps2):
        dt = self.dtype
        t = lambda k: torch.as_tensor(batch[k]).to(dt)
        obs, actions, next_obs = t("observations"), t("actions"), t("next_observations")
        rewards, terminals = t("rewards"), t("terminals")
        eps1, eps2 = torch.as_tensor(eps1).to(dt), torch.as_tensor(eps2).to(dt)
        # policy and alpha loss                                   trainer.py:136-149
        new_actions, mean, log_std, log_pi = self.policy.policy(obs, eps1)
        if self.auto_alpha:
            alpha_loss = -(self.log_alpha * (log_pi + self.target_entropy).detach()).mean()
            self.alpha_optimizer.zero_grad()
            alpha_loss.backward()
            self.alpha_optimizer.step()
            alpha = self.log_alpha.exp()
        else:
            alpha_loss, alpha = torch.zeros(()), 0
        q_new = torch.min(self.qf1.q(obs, new_actions), self.qf2.q(obs, new_actions))   # :151-154
        policy_loss = (alpha * log_pi - q_new).mean()                                   # :160
        # critic loss                                             trainer.py:168-196
        q1_pred, q2_pred = self.qf1.q(obs, actions), self.qf2.q(obs, actions)
        next_actions, _, _, new_log_pi = self.policy.policy(next_obs, eps2)
        target_q = torch.min(self.target_qf1.q(next_obs, next_actions),
                             self.target_qf2.q(next_obs, next_actions)) - alpha * new_log_pi
        q_target = self.reward_scale * rewards + (1.0 - terminals) * self.discount * target_q
        qf1_loss = ((q1_pred - q_target.detach()) ** 2).mean()
        qf2_loss = ((q2_pred - q_target.detach()) ** 2).mean()
        # updates, in the reference's order                       trainer.py:200-210
        self.qf1_optimizer.zero_grad()
        qf1_loss.backward()
        g1 = {k: p.grad.clone() for k, p in self.qf1.named().items()}
        self.qf1_optimizer.step()
        self.qf2_optimizer.zero_grad()
        qf2_loss.backward()
        g2 = {k: p.grad.clone() for k, p in self.qf2.named().items()}
        self.qf2_optimizer.step()
        self.policy_optimizer.zero_grad()
        policy_loss.backward()   # through the post-step critics (quirk Q1)
        gp = {k: p.grad.clone() for k, p in self.policy.named().items()}
        self.policy_optimizer.step()
        # Polyak                                                   trainer.py:215-224
        if self.n_steps % self.period == 0:
            with torch.no_grad():
                for src, dst in ((self.qf1, self.target_qf1), (self.qf2, self.target_qf2)):
                    for ps, pt in zip(src.parameters(), dst.parameters()):
                        pt.data.copy_(pt.data * (1.0 - self.tau) + ps.data * self.tau)
        self.n_steps += 1
        return dict(grads=dict(policy=gp, qf1=g1, qf2=g2), qf1_loss=qf1_loss.detach(),
                    qf2_loss=qf2_loss.detach(), policy_loss=policy_loss.detach(),
                    alpha_loss=torch.as_tensor(alpha_loss).detach())

    def state(self):
        """{group: {reference key: tensor}} of the post-step parameters."""
        return {g: {k: p.detach() for k, p in getattr(self, g).named().items()}
                for g in ("policy", "qf1", "qf2", "target_qf1", "target_qf2")}


class ParticleOACAutograd:
    """ParticleTrainer of trainer/particle_trainer_oac.py (share_layers=True:
    one critic with K outputs, the P-OAC trainer of BASELINE configs[4]) on
    torch autograd, CPU -- the reference's op sequence of train_from_torch
    (lines 169-324) for the configs[4] CPU baseline:

    * critic on (obs, a), permute to [K, B, 1], torch.sort over K     :185-192
    * policy(next_obs) (eps1), target critic, sort, quantile target   :193-208
    * counts=True re-centring of drawn rows                          :220-224
    * the K MSEs summed (not averaged), one backward, Adam             :247-256
    * policy(obs) (eps2) after the critic step, alpha loss and step   :271-284
    * the post-step critic on (obs, a~), sort, policy loss on slot 0  :286-300
    * Polyak                                                           :320-324

    As in the reference, the policy backward also runs through (and
    accumulates into) the critic's parameters, whose grads the next step's
    zero_grad drops."""

    def __init__(self, params, obs_dim, act_dim, K, discount=0.99, reward_scale=1.0,
                 policy_lr=3e-4, qf_lr=3e-4, tau=5e-3, target_update_period=1,
                 target_entropy=None, dtype=torch.float32):
        self.dtype, self.K = dtype, K
        self.policy = _Mlp(params["policy"], dtype, policy=True)
        self.qf = _Mlp(params["qf1"], dtype)
        self.tf = _Mlp(params["target_qf1"], dtype)
        self.discount, self.reward_scale, self.tau = discount, reward_scale, tau
        self.period = target_update_period
        self.target_entropy = -float(act_dim) if target_entropy is None else target_entropy
        self.log_alpha = torch.zeros(1, dtype=dtype, requires_grad=True)
        self.qf_optimizer = Adam14(self.qf.parameters(), qf_lr)
        self.policy_optimizer = Adam14(self.policy.parameters(), policy_lr)
        self.alpha_optimizer = Adam14([self.log_alpha], policy_lr)
        self.n_steps = 0

    def step(self, batch, eps1, eps2):
        dt = self.dtype
        t = lambda k: torch.as_tensor(batch[k]).to(dt)
        obs, actions, next_obs = t("observations"), t("actions"), t("next_observations")
        rewards, terminals = t("rewards"), t("terminals")
        eps1, eps2 = torch.as_tensor(eps1).to(dt), torch.as_tensor(eps2).to(dt)
        qs = torch.stack([self.qf.q(obs, actions)], dim=0).permute(2, 1, 0)      # [K, B, 1]
        sorted_qs, _ = torch.sort(qs, dim=0)
        next_actions, _, _, _ = self.policy.policy(next_obs, eps1)
        target_qs = torch.stack([self.tf.q(next_obs, next_actions)], dim=0).permute(2, 1, 0)
        target_sorted, _ = torch.sort(target_qs, dim=0)
        q_target = self.reward_scale * rewards + (1.0 - terminals) * self.discount * target_sorted
        if batch.get("counts") is not None:
            counts = t("counts")
            factor = torch.zeros_like(counts)
            factor[counts == 0] = 1
            q_target = (q_target * factor) + (1 - factor) * (
                sorted_qs - torch.mean(sorted_qs, dim=0) + torch.mean(q_target, dim=0))
        qf_losses, qf_loss = [], 0
        for i in range(self.K):
            q_loss = ((sorted_qs[i] - q_target[i].detach()) ** 2).mean()
            qf_losses.append(q_loss)
            qf_loss = qf_loss + q_loss
        self.qf_optimizer.zero_grad()
        qf_loss.backward(retain_graph=True)
        gq = {k: p.grad.clone() for k, p in self.qf.named().items()}
        self.qf_optimizer.step()
        new_actions, mean, log_std, log_pi = self.policy.policy(obs, eps2)
        alpha_loss = -(self.log_alpha * (log_pi + self.target_entropy).detach()).mean()
        self.alpha_optimizer.zero_grad()
        alpha_loss.backward()
        g_la = self.log_alpha.grad.clone()   # (the policy backward adds to it later)
        self.alpha_optimizer.step()
        alpha = self.log_alpha.exp()
        pi_qs = torch.stack([self.qf.q(obs, new_actions)], dim=0).permute(2, 1, 0)
        q_new = torch.sort(pi_qs, dim=0)[0][0]
        policy_loss = (alpha * log_pi - q_new).mean()
        self.policy_optimizer.zero_grad()
        policy_loss.backward()
        gp = {k: p.grad.clone() for k, p in self.policy.named().items()}
        self.policy_optimizer.step()
        if self.n_steps % self.period == 0:
            with torch.no_grad():
                for ps, pt in zip(self.qf.parameters(), self.tf.parameters()):
                    pt.data.copy_(pt.data * (1.0 - self.tau) + ps.data * self.tau)
        self.n_steps += 1
        return dict(grads=dict(policy=gp, qf=gq, log_alpha=g_la),
                    qf_losses=torch.stack([q.detach() for q in qf_losses]),
                    policy_loss=policy_loss.detach(), alpha_loss=alpha_loss.detach())

    def state(self):
        return {g: {k: p.detach() for k, p in m.named().items()}
                for g, m in (("policy", self.policy), ("qf", self.qf), ("tf", self.tf))}
