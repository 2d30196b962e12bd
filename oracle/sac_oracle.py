"""CPU restatement of the reference's SAC / OAC / P-OAC hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``oac-explore_amd/``) may
import this module: it is the checker the parity tests compare the HIP path
against, and the ``cpu_baseline`` leg that ``bench.py`` times on the host.

It restates, with explicit forward and backward passes written out by hand
(no autograd), the semantics of:

* ``ReplayBuffer.random_batch``        /root/reference/replay_buffer.py:106-115
* ``np_to_pytorch_batch``              /root/reference/utils/core.py:40-61
* ``Mlp.forward`` / ``FlattenMlp``     /root/reference/networks.py:62-79,159-161
* ``TanhGaussianPolicy.forward``       /root/reference/trainer/policies.py:260-316
* ``TanhNormal.log_prob / rsample``    /root/reference/trainer/policies.py:147-160,175-192
* ``SACTrainer.train_from_torch``      /root/reference/trainer/trainer.py:126-280
  with the torch-1.4 update order (the policy
  gradient back-propagates through the POST-step Q weights with the PRE-step
  activations / ReLU masks);
* ``ParticleTrainer.train_from_torch`` /root/reference/trainer/particle_trainer_oac.py:169-363
  (shared-layer K-head critic);
* ``GaussianTrainer.train_from_torch`` /root/reference/trainer/gaussian_trainer.py:177-437
  (g-oac: shared-layer critic with outputs [Q | log std], deterministic
  policy, separately trained target_policy);
* ``ParticleTrainer.train_from_torch`` /root/reference/trainer/particle_trainer.py:175-432
  (the p-oac recipes: K-particle critic, deterministic policy, upper-bound
  quantile policy loss, target_policy);
* ``get_optimistic_exploration_action_stochastic``
                                       /root/reference/optimistic_exploration.py:14-109
* torch 1.4 ``optim.Adam.step`` (constructed at trainer/trainer.py:75-91) and
  ``soft_update_from_to``              /root/reference/utils/pytorch_util.py:5-9

Pinned against golden vectors produced by running the reference itself in the
build container (tests/golden/make_golden.py -> tests/golden/*.npz); see
tests/test_oracle_golden.py.

Everything computes in ``dtype`` (float32 by default, like the reference;
float64 is used by the tests to measure the fp32 noise floor).
"""
import math

import numpy as np
import torch

LOG_SIG_MAX = 2.0    # trainer/policies.py:10
LOG_SIG_MIN = -20.0  # trainer/policies.py:11
TANH_EPS = 1e-6      # TanhNormal(epsilon=1e-6), trainer/policies.py:127
HALF_LOG_2PI = math.log(math.sqrt(2 * math.pi))  # torch Normal.log_prob constant


# --------------------------------------------------------------- helpers
def _t(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(dtype)
    return torch.from_numpy(np.ascontiguousarray(x)).to(dtype)


def to_torch_params(d, dtype=torch.float32):
    return {k: _t(v, dtype).clone() for k, v in d.items()}


def linear(x, W, b):
    """nn.Linear as torch 1.4 ran it: addmm(b, x, W.t())  (networks.py:65)."""
    return torch.addmm(b, x, W.t())


def n_hidden(p):
    return sum(1 for k in p if k.startswith("fc") and k.endswith(".weight"))


# ------------------------------------------------------------- networks
def mlp_trunk(x, p):
    """Hidden stack of Mlp.forward (networks.py:63-66): relu(fc_i(h))."""
    hs = [x]
    h = x
    for i in range(n_hidden(p)):
        h = torch.relu(linear(h, p[f"fc{i}.weight"], p[f"fc{i}.bias"]))
        hs.append(h)
    return hs


def q_forward(obs, act, p):
    """FlattenMlp.forward (networks.py:159-161 -> 62-79), identity output."""
    x = torch.cat([obs, act], dim=1)
    hs = mlp_trunk(x, p)
    q = linear(hs[-1], p["last_fc.weight"], p["last_fc.bias"])
    return dict(hs=hs, q=q)


def q_param_grads(cache, dq, p):
    """Gradient of sum(dq * Q(x)) w.r.t. every Q parameter (MSE backward
    through Mlp.forward)."""
    hs = cache["hs"]
    L = len(hs) - 1
    g = {}
    g["last_fc.weight"] = dq.t() @ hs[L]
    g["last_fc.bias"] = dq.sum(0)
    dh = (dq @ p["last_fc.weight"]) * (hs[L] > 0)
    for i in range(L - 1, -1, -1):
        g[f"fc{i}.weight"] = dh.t() @ hs[i]
        g[f"fc{i}.bias"] = dh.sum(0)
        if i > 0:
            dh = (dh @ p[f"fc{i}.weight"]) * (hs[i] > 0)
    return g


def q_input_grad(cache, dq, p):
    """d sum(dq*Q)/d x, using the weights in ``p`` and the masks saved in
    ``cache`` (this is how the torch-1.4 quirk enters: p = post-step)."""
    hs = cache["hs"]
    L = len(hs) - 1
    dh = (dq @ p["last_fc.weight"]) * (hs[L] > 0)
    for i in range(L - 1, -1, -1):
        dh = dh @ p[f"fc{i}.weight"]
        if i > 0:
            dh = dh * (hs[i] > 0)
    return dh


def policy_forward(obs, p, eps, deterministic=False):
    """TanhGaussianPolicy.forward(reparameterize=True, return_log_prob=True)
    (policies.py:272-304) with TanhNormal.rsample / log_prob (175-192, 147-160);
    ``eps`` is the standard-normal draw of ``Normal(0,1).sample()`` (183-185)."""
    hs = mlp_trunk(obs, p)
    h = hs[-1]
    mean = linear(h, p["last_fc.weight"], p["last_fc.bias"])
    ls_raw = linear(h, p["last_fc_log_std.weight"], p["last_fc_log_std.bias"])
    log_std = torch.clamp(ls_raw, LOG_SIG_MIN, LOG_SIG_MAX)
    std = torch.exp(log_std)
    if deterministic:
        a = torch.tanh(mean)
        return dict(hs=hs, mean=mean, ls_raw=ls_raw, log_std=log_std, std=std, a=a,
                    z=mean, logp=torch.zeros_like(a), eps=None)
    z = mean + std * eps
    a = torch.tanh(z)
    var = std ** 2
    u = z - mean
    lp = -(u ** 2) / (2 * var) - torch.log(std) - HALF_LOG_2PI \
        - torch.log(1 - a * a + TANH_EPS)
    logp = lp.sum(dim=1, keepdim=True)
    return dict(hs=hs, mean=mean, ls_raw=ls_raw, log_std=log_std, std=std, a=a, z=z,
                logp=logp, eps=eps, u=u, var=var)


def policy_head_grads(c, ga, G):
    """Upstream gradients on the two heads' outputs (mean, raw log_std) of
    sum(ga * a) + sum(G * logp): policies.py:154-160,179-190,275-279 (clamp
    passes the gradient where LOG_SIG_MIN <= x <= LOG_SIG_MAX)."""
    a, std, u, var, eps = c["a"], c["std"], c["u"], c["var"], c["eps"]
    da = ga + G * (2 * a / (1 - a * a + TANH_EPS))
    dz = da * (1 - a * a) - G * (u / var)
    dmean = dz + G * (u / var)
    dstd = dz * eps + G * (u * u * std / (var * var) - 1.0 / std)
    dls = dstd * std
    dls = dls * ((c["ls_raw"] >= LOG_SIG_MIN) & (c["ls_raw"] <= LOG_SIG_MAX))
    return dmean, dls


def policy_backward(c, p, ga, G):
    """Gradients of  sum(ga * a) + sum(G * logp)  w.r.t. the policy params.

    ga: [B,Da] upstream grad on the tanh action, G: [B,1] upstream grad on
    log_prob (policy_head_grads), then the trunk's backward."""
    dmean, dls = policy_head_grads(c, ga, G)
    hs = c["hs"]
    L = len(hs) - 1
    g = {}
    g["last_fc.weight"] = dmean.t() @ hs[L]
    g["last_fc.bias"] = dmean.sum(0)
    g["last_fc_log_std.weight"] = dls.t() @ hs[L]
    g["last_fc_log_std.bias"] = dls.sum(0)
    dh = (dmean @ p["last_fc.weight"] + dls @ p["last_fc_log_std.weight"]) * (hs[L] > 0)
    for i in range(L - 1, -1, -1):
        g[f"fc{i}.weight"] = dh.t() @ hs[i]
        g[f"fc{i}.bias"] = dh.sum(0)
        if i > 0:
            dh = (dh @ p[f"fc{i}.weight"]) * (hs[i] > 0)
    return g


# ------------------------------------------------------- optimiser / target
class Adam14:
    """torch 1.4.0 optim.Adam.step (no weight decay, no amsgrad)."""

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8):
        self.p = params
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.t = 0

    def step(self, grads):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for k, g in grads.items():
            m, v = self.m[k], self.v[k]
            m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            self.p[k].addcdiv_(m, denom, value=-(self.lr / bc1))


def polyak(target, source, tau):
    """soft_update_from_to (utils/pytorch_util.py:5-9)."""
    for k in target:
        target[k].copy_(target[k] * (1.0 - tau) + source[k] * tau)


# ---------------------------------------------------------------- replay
class NumpyReplay:
    """Host float64 ring buffer + uniform gather (replay_buffer.py:32-48,88-115)
    and the numpy->fp32 batch conversion (utils/core.py:40-61)."""

    def __init__(self, data):
        self.d = {k: np.asarray(v) for k, v in data.items()}
        self.size = len(self.d["observations"])

    def random_batch(self, B, rs=None):
        idx = (rs or np.random).randint(0, self.size, B)
        return idx, {k: v[idx] for k, v in self.d.items()}

    @staticmethod
    def to_torch(batch, dtype=torch.float32):
        return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in batch.items()}


# ------------------------------------------------------------------- SAC
class SACOracle:
    """SACTrainer.train_from_torch (trainer/trainer.py:126-280)."""

    def __init__(self, params, obs_dim, act_dim, discount=0.99, reward_scale=1.0,
                 policy_lr=3e-4, qf_lr=3e-4, tau=5e-3, target_update_period=1,
                 auto_alpha=True, target_entropy=None, log_alpha0=0.0,
                 dtype=torch.float32):
        self.dtype = dtype
        self.Do, self.Da = obs_dim, act_dim
        self.P = to_torch_params(params["policy"], dtype)
        self.Q1 = to_torch_params(params["qf1"], dtype)
        self.Q2 = to_torch_params(params["qf2"], dtype)
        self.T1 = to_torch_params(params["target_qf1"], dtype)
        self.T2 = to_torch_params(params["target_qf2"], dtype)
        self.discount, self.reward_scale, self.tau = discount, reward_scale, tau
        self.period = target_update_period
        self.auto_alpha = auto_alpha
        self.target_entropy = -float(act_dim) if target_entropy is None else target_entropy
        self.log_alpha = torch.full((1,), log_alpha0, dtype=dtype)
        self.opt_p = Adam14(self.P, policy_lr)
        self.opt_q1 = Adam14(self.Q1, qf_lr)
        self.opt_q2 = Adam14(self.Q2, qf_lr)
        self.opt_a = Adam14({"log_alpha": self.log_alpha}, policy_lr)
        self.n_steps = 0
        self.last = {}

    # The step is written as four phases separated by the only points where a
    # whole-batch quantity is needed; the single-process step runs them back
    # to back, the data-parallel test all-reduces alpha_sum / crit_flat /
    # pol_flat (SUM) between them (oac_amd/dp.py).
    def step(self, batch, eps1, eps2):
        self.phase0(batch, eps1, eps2)
        self.phase1()
        self.phase2()
        return self.phase3()

    def _flat(self, grads, order):
        flat = torch.cat([grads[k].reshape(-1) for k in order])
        views, o = {}, 0
        for k in order:
            n = grads[k].numel()
            views[k] = flat[o:o + n].view(grads[k].shape)
            o += n
        return flat, views

    def phase0(self, batch, eps1, eps2):
        dt = self.dtype
        S = self.S = {}
        S["obs"] = _t(batch["observations"], dt)
        S["act"] = _t(batch["actions"], dt)
        S["rew"] = _t(batch["rewards"], dt)
        S["term"] = _t(batch["terminals"], dt)
        S["nobs"] = _t(batch["next_observations"], dt)
        S["B"] = S["obs"].shape[0]
        # E1  policy(obs)                                        trainer.py:136-138
        S["pf"] = policy_forward(S["obs"], self.P, _t(eps1, dt))
        # E4                                                     trainer.py:168-169
        S["c1"] = q_forward(S["obs"], S["act"], self.Q1)
        S["c2"] = q_forward(S["obs"], S["act"], self.Q2)
        # E5                                                     trainer.py:172-174
        S["pf2"] = policy_forward(S["nobs"], self.P, _t(eps2, dt))
        # local sum(logp + H) for the alpha gradient
        self.alpha_sum = (S["pf"]["logp"] + self.target_entropy).sum(0)

    def phase1(self, world=1):
        S, dt = self.S, self.dtype
        B = S["B"]
        pf, pf2 = S["pf"], S["pf2"]
        # E2  alpha                                              trainer.py:139-149
        if self.auto_alpha:
            n = B * world
            g_la = -(self.alpha_sum / n)
            alpha_loss = -(self.log_alpha * self.alpha_sum) / n
            self.opt_a.step({"log_alpha": g_la})
            alpha = self.log_alpha.exp()
        else:
            g_la, alpha_loss, alpha = None, torch.zeros(()), torch.zeros(1, dtype=dt)
        S.update(g_la=g_la, alpha_loss=alpha_loss, alpha=alpha)
        # E3  min Q on the fresh actions (pre-step weights)      trainer.py:151-160
        S["c1n"] = q_forward(S["obs"], pf["a"], self.Q1)
        S["c2n"] = q_forward(S["obs"], pf["a"], self.Q2)
        S["q_new"] = torch.min(S["c1n"]["q"], S["c2n"]["q"])
        S["policy_loss"] = (alpha * pf["logp"] - S["q_new"]).mean()
        # E6                                                     trainer.py:178-184
        t1 = q_forward(S["nobs"], pf2["a"], self.T1)["q"]
        t2 = q_forward(S["nobs"], pf2["a"], self.T2)["q"]
        target_q = torch.min(t1, t2) - alpha * pf2["logp"]
        y = self.reward_scale * S["rew"] + (1.0 - S["term"]) * self.discount * target_q
        S["y"] = y
        # E7                                                     trainer.py:194-196
        c1, c2 = S["c1"], S["c2"]
        S["qf1_loss"] = ((c1["q"] - y) ** 2).mean()
        S["qf2_loss"] = ((c2["q"] - y) ** 2).mean()
        g1 = q_param_grads(c1, 2.0 * (c1["q"] - y) / B, self.Q1)
        g2 = q_param_grads(c2, 2.0 * (c2["q"] - y) / B, self.Q2)
        order = list(self.Q1.keys())
        self.crit_flat, views = self._flat({**{"1/" + k: g1[k] for k in order},
                                            **{"2/" + k: g2[k] for k in order}},
                                           ["1/" + k for k in order] + ["2/" + k for k in order])
        S["g1"] = {k: views["1/" + k] for k in order}
        S["g2"] = {k: views["2/" + k] for k in order}

    def phase2(self, world=1):
        S, pf = self.S, self.S["pf"]
        B = S["B"]
        # E8  Q1 step, Q2 step, then the policy backward          trainer.py:200-210
        self.opt_q1.step({k: v / world for k, v in S["g1"].items()})
        self.opt_q2.step({k: v / world for k, v in S["g2"].items()})
        c1n, c2n = S["c1n"], S["c2n"]
        sel1 = (c1n["q"] <= c2n["q"]).to(self.dtype)   # torch-1.4 min() backward
        gq = -torch.ones_like(S["q_new"]) / B
        Do = self.Do
        da = q_input_grad(c1n, gq * sel1, self.Q1)[:, Do:] \
            + q_input_grad(c2n, gq * (1 - sel1), self.Q2)[:, Do:]
        G = (S["alpha"] / B) * torch.ones_like(pf["logp"])
        S["pol_up"] = (da, G)   # the policy backward's upstream gradients (parity checks)
        gp = policy_backward(pf, self.P, da, G)
        order = list(self.P.keys())
        self.pol_flat, views = self._flat(gp, order)
        S["gp"] = views
        # E9  Polyak (uses only the post-step critics)            trainer.py:215-224
        if self.n_steps % self.period == 0:
            polyak(self.T1, self.Q1, self.tau)
            polyak(self.T2, self.Q2, self.tau)

    def phase3(self, world=1):
        S = self.S
        self.opt_p.step({k: v / world for k, v in S["gp"].items()})
        stats = self._stats(S["c1"]["q"], S["c2"]["q"], S["y"], S["pf"], S["q_new"],
                            S["qf1_loss"], S["qf2_loss"], S["alpha"], S["alpha_loss"])
        self.n_steps += 1
        self.last = dict(grads=dict(policy=S["gp"], qf1=S["g1"], qf2=S["g2"],
                                    log_alpha=S["g_la"]),
                         qf1_loss=S["qf1_loss"], qf2_loss=S["qf2_loss"],
                         policy_loss=S["policy_loss"], alpha=S["alpha"],
                         alpha_loss=S["alpha_loss"], y=S["y"], q1=S["c1"]["q"],
                         q2=S["c2"]["q"], logp=S["pf"]["logp"], logp2=S["pf2"]["logp"],
                         a=S["pf"]["a"], a2=S["pf2"]["a"], stats=stats,
                         pf=S["pf"], pol_up=S["pol_up"])
        return self.last

    def _stats(self, q1, q2, y, pf, q_new, l1, l2, alpha, alpha_loss):
        """eval_statistics keys of trainer.py:243-279 (Q5: 'Policy Loss' is
        recomputed without alpha, :236)."""
        n = lambda t: t.detach().to(torch.float32).numpy()
        st = {}
        qs = np.stack([n(q1), n(q2)], 0)
        st["QF mean"] = np.mean(qs, axis=0).mean()
        st["QF std"] = np.std(qs, axis=0).mean()
        st["QF1 Loss"] = float(l1)
        st["QF2 Loss"] = float(l2)
        st["Q Loss"] = float(l1 + l2)
        st["Policy Loss"] = float((pf["logp"] - q_new).mean())
        for name, arr in (("Q1 Predictions", q1), ("Q2 Predictions", q2), ("Q Targets", y),
                          ("Log Pis", pf["logp"]), ("Policy mu", pf["mean"]),
                          ("Policy log std", pf["log_std"])):
            a = n(arr)
            st[name + " Mean"] = np.mean(a)
            st[name + " Std"] = np.std(a)
            st[name + " Max"] = np.max(a)
            st[name + " Min"] = np.min(a)
        if self.auto_alpha:
            st["Alpha"] = float(alpha)
            st["Alpha Loss"] = float(alpha_loss)
        return st


# ----------------------------------------------------------------- P-OAC
class ParticleOACOracle:
    """ParticleTrainer (particle_trainer_oac.py) with share_layers=True: one
    critic with K outputs, per-sample sort over K (lines 169-363)."""

    def __init__(self, params, obs_dim, act_dim, K, discount=0.99, reward_scale=1.0,
                 policy_lr=3e-4, qf_lr=3e-4, tau=5e-3, target_update_period=1,
                 target_entropy=None, train_bias=True, dtype=torch.float32):
        self.dtype = dtype
        self.train_bias = train_bias
        self.Do, self.Da, self.K = obs_dim, act_dim, K
        self.P = to_torch_params(params["policy"], dtype)
        self.Q = to_torch_params(params["qf1"], dtype)
        self.T = to_torch_params(params["target_qf1"], dtype)
        self.discount, self.reward_scale, self.tau = discount, reward_scale, tau
        self.period = target_update_period
        self.target_entropy = -float(act_dim) if target_entropy is None else target_entropy
        self.log_alpha = torch.zeros(1, dtype=dtype)
        self.opt_p = Adam14(self.P, policy_lr)
        self.opt_q = Adam14(self.Q, qf_lr)
        self.opt_a = Adam14({"log_alpha": self.log_alpha}, policy_lr)
        self.n_steps = 0

    def step(self, batch, eps1, eps2):
        dt = self.dtype
        obs = _t(batch["observations"], dt)
        act = _t(batch["actions"], dt)
        rew = _t(batch["rewards"], dt)
        term = _t(batch["terminals"], dt)
        nobs = _t(batch["next_observations"], dt)
        eps1, eps2 = _t(eps1, dt), _t(eps2, dt)
        B = obs.shape[0]
        c = q_forward(obs, act, self.Q)                      # lines 185-191
        qs = c["q"].t()                                      # [K,B]
        sorted_qs, qs_idx = torch.sort(qs, dim=0)            # line 192
        pf2 = policy_forward(nobs, self.P, eps1)             # 193-195
        tq = q_forward(nobs, pf2["a"], self.T)["q"].t()      # 198-201
        tq_sorted, _ = torch.sort(tq, dim=0)                 # 202
        y = self.reward_scale * rew.t() + (1.0 - term.t()) * self.discount * tq_sorted  # 207-208
        if batch.get("counts") is not None:                  # counts=True, 220-224
            cnt = _t(batch["counts"], dt).reshape(1, B)
            factor = (cnt == 0).to(dt)
            y = y * factor + (1 - factor) * (sorted_qs - sorted_qs.mean(dim=0) + y.mean(dim=0))
        losses = ((sorted_qs - y) ** 2).mean(dim=1)          # 247-251
        d_sorted = 2.0 * (sorted_qs - y) / B
        dq = torch.zeros_like(qs).scatter_(0, qs_idx, d_sorted).t()   # sort backward
        gq = q_param_grads(c, dq, self.Q)
        if not self.train_bias:                              # frozen last bias (networks.py:59-60)
            gq["last_fc.bias"] = torch.zeros_like(gq["last_fc.bias"])
        self.opt_q.step(gq)                                  # 252-256
        pf = policy_forward(obs, self.P, eps2)               # 271-273
        w = pf["logp"] + self.target_entropy                 # 274-281
        g_la = (-(w / B)).sum(0)
        alpha_loss = -(self.log_alpha * w).mean()
        self.opt_a.step({"log_alpha": g_la})
        alpha = self.log_alpha.exp()
        cn = q_forward(obs, pf["a"], self.Q)                 # 286 (post-step Q)
        pq = cn["q"].t()
        sq, sidx = torch.sort(pq, dim=0)                     # 291
        q_new = sq[0]
        policy_loss = (alpha * pf["logp"][:, 0] - q_new).mean()
        gsel = torch.zeros_like(pq).scatter_(0, sidx[:1], -torch.ones_like(q_new)[None] / B).t()
        da = q_input_grad(cn, gsel, self.Q)[:, self.Do:]
        G = (alpha / B) * torch.ones_like(pf["logp"])
        gp = policy_backward(pf, self.P, da, G)
        self.opt_p.step(gp)                                  # 298-300
        if self.n_steps % self.period == 0:                  # 320-324
            polyak(self.T, self.Q, self.tau)
        self.n_steps += 1
        self.last = dict(grads=dict(policy=gp, qf=gq, log_alpha=g_la), qf_losses=losses,
                         qf_loss=losses.sum(), policy_loss=policy_loss, alpha=alpha,
                         alpha_loss=alpha_loss, sorted_qs=sorted_qs, y=y, tq=tq,
                         policy_mean=pf["mean"], policy_log_std=pf["log_std"],
                         pf=pf, pol_up=(da, G))
        return self.last


def det_policy_backward(c, p, ga):
    """Gradient of sum(ga * tanh(mean)) w.r.t. the params of a deterministic
    TanhGaussianPolicy (policies.py:286-288); the log-std head is not in the
    graph (zeros here; torch Adam skips it, which leaves it unchanged too)."""
    a, hs = c["a"], c["hs"]
    dmean = ga * (1 - a * a)
    L = len(hs) - 1
    g = {"last_fc.weight": dmean.t() @ hs[L], "last_fc.bias": dmean.sum(0),
         "last_fc_log_std.weight": torch.zeros_like(p["last_fc_log_std.weight"]),
         "last_fc_log_std.bias": torch.zeros_like(p["last_fc_log_std.bias"])}
    dh = (dmean @ p["last_fc.weight"]) * (hs[L] > 0)
    for i in range(L - 1, -1, -1):
        g[f"fc{i}.weight"] = dh.t() @ hs[i]
        g[f"fc{i}.bias"] = dh.sum(0)
        if i > 0:
            dh = (dh @ p[f"fc{i}.weight"]) * (hs[i] > 0)
    return g


class GaussianOACOracle:
    """GaussianTrainer (gaussian_trainer.py) with share_layers=True and the
    deterministic policy (the reproduce_g-oac*.sh configuration): critic Q
    with raw outputs [mean | log std] (FlattenMlp positive=[False, True],
    networks.py:69-75), target critic, policy and target_policy."""

    def __init__(self, params, obs_dim, act_dim, delta=0.95, q_min=0.0, q_max=100.0,
                 discount=0.99, reward_scale=1.0, policy_lr=3e-4, qf_lr=3e-4, tau=5e-3,
                 target_update_period=1, std_soft_update_prob=None, mean_update=False,
                 train_bias=True, next_policy=None, dtype=torch.float32):
        from scipy.stats import norm
        self.mean_update = mean_update
        self.train_bias = train_bias
        self.dtype = dtype
        self.Do, self.Da = obs_dim, act_dim
        self.P = to_torch_params(params["policy"], dtype)
        self.TP = to_torch_params(params["target_policy"], dtype)
        # use_target_policy (gaussian_trainer.py:154-158, particle_trainer.py:
        # 150-154): the DDPG target network acts on next_obs; its soft update
        # copies it onto itself (:385-387), so its weights never change
        self.NP = None if next_policy is None else to_torch_params(next_policy, dtype)
        self.Q = to_torch_params(params["qf1"], dtype)
        self.T = to_torch_params(params["target_qf1"], dtype)
        self.z = float(norm.ppf(delta, loc=0, scale=1))          # gaussian_trainer.py:69
        self.std_init = (q_max - q_min) / np.sqrt(12)            # :72
        self.discount, self.reward_scale, self.tau = discount, reward_scale, tau
        self.period = target_update_period
        self.soft = std_soft_update_prob
        self.opt_p = Adam14(self.P, policy_lr)
        self.opt_tp = Adam14(self.TP, policy_lr)
        self.opt_q = Adam14(self.Q, qf_lr)
        self.n_steps = 0

    def step(self, batch):
        self.phase0(batch)
        self.phase1()
        self.phase2()
        return self.phase3()

    def _next_policy(self):
        """The policy acting on next_obs: target_policy with mean_update, else
        the DDPG target network with use_target_policy, else the policy
        (gaussian_trainer.py:194-205, particle_trainer.py:194-205)."""
        if self.mean_update:
            return self.TP
        return self.NP if self.NP is not None else self.P

    @staticmethod
    def _flat(grads, order):
        return torch.cat([grads[k].reshape(-1) for k in order])

    @staticmethod
    def _unflat(flat, like, order):
        out, o = {}, 0
        for k in order:
            n = like[k].numel()
            out[k] = flat[o:o + n].view(like[k].shape)
            o += n
        return out

    # data-parallel split (oac_amd.dp.dp_step): the only cross-rank quantities
    # are the critic and the policy gradients (local batch means; the Adam
    # passes divide the all-reduced sums by the world size)
    def phase0(self, batch):
        dt = self.dtype
        S = self.S = {}
        obs = S["obs"] = _t(batch["observations"], dt)
        act = _t(batch["actions"], dt)
        rew = _t(batch["rewards"], dt)
        term = _t(batch["terminals"], dt)
        nobs = _t(batch["next_observations"], dt)
        B = S["B"] = obs.shape[0]
        c = S["c"] = q_forward(obs, act, self.Q)                     # :187
        q_preds, std_preds = c["q"][:, :1], torch.exp(c["q"][:, 1:2])
        pf2 = policy_forward(nobs, self._next_policy(), None, deterministic=True)   # :192-202
        tq = q_forward(nobs, pf2["a"], self.T)["q"]                  # :204
        tq0, tstd = tq[:, :1], torch.exp(tq[:, 1:2])
        std_target = (1. - term) * self.discount * tstd              # :213
        if self.soft is not None:                                    # :215-218
            std_target = self.soft * std_target + (1 - self.soft) * std_preds
        if batch.get("counts") is not None:                          # :220-224
            cnt = _t(batch["counts"], dt).reshape(B, 1)
            factor = (cnt == 0).to(dt)
            std_target = std_target * factor + (1 - factor) * std_preds
        q_target = self.reward_scale * rew + (1. - term) * self.discount * tq0   # :227-228
        std_target = torch.clamp(std_target, 0, self.std_init)       # :229
        S.update(q_preds=q_preds, std_preds=std_preds, q_target=q_target, std_target=std_target,
                 q_loss=((q_preds - q_target) ** 2).mean(),          # :231-234
                 std_loss=((std_preds - std_target) ** 2).mean())
        # both policy forwards on obs use the pre-step policies      :315-318, :342-344
        S["pf"] = policy_forward(obs, self.P, None, deterministic=True)
        S["tpf"] = policy_forward(obs, self.TP, None, deterministic=True)

    def phase1(self, world=1):
        S = self.S
        B = S["B"]
        dq = torch.cat([2.0 * (S["q_preds"] - S["q_target"]) / B,
                        2.0 * (S["std_preds"] - S["std_target"]) / B * S["std_preds"]], dim=1)
        S["gq"] = q_param_grads(S["c"], dq, self.Q)
        if not self.train_bias:                              # frozen last bias (networks.py:59-60)
            S["gq"]["last_fc.bias"] = torch.zeros_like(S["gq"]["last_fc.bias"])
        self.crit_flat = self._flat(S["gq"], list(self.Q))

    def phase2(self, world=1):
        S = self.S
        B, obs = S["B"], S["obs"]
        gq = self._unflat(self.crit_flat, self.Q, list(self.Q))
        self.opt_q.step({k: v / world for k, v in gq.items()})     # :237
        pf, tpf = S["pf"], S["tpf"]
        cn = q_forward(obs, pf["a"], self.Q)                         # :325 (post-step Q)
        qs, stds = cn["q"][:, :1], torch.exp(cn["q"][:, 1:2])
        S["ub"] = qs + self.z * stds                                 # :331
        g0 = -torch.ones_like(qs) / B
        da = q_input_grad(cn, torch.cat([g0, g0 * self.z * stds], dim=1), self.Q)[:, self.Do:]
        S["gp"] = det_policy_backward(pf, self.P, da)
        ct = q_forward(obs, tpf["a"], self.Q)                        # :346
        dat = q_input_grad(ct, torch.cat([g0, torch.zeros_like(g0)], dim=1), self.Q)[:, self.Do:]
        S["gtp"] = det_policy_backward(tpf, self.TP, dat)
        self.pol_flat = torch.cat([self._flat(S["gp"], list(self.P)),
                                   self._flat(S["gtp"], list(self.TP))])

    def phase3(self, world=1):
        S = self.S
        n = self._flat(S["gp"], list(self.P)).numel()
        gp = self._unflat(self.pol_flat[:n], self.P, list(self.P))
        gtp = self._unflat(self.pol_flat[n:], self.TP, list(self.TP))
        self.opt_p.step({k: v / world for k, v in gp.items()})      # :334-337
        self.opt_tp.step({k: v / world for k, v in gtp.items()})    # :352-354
        if self.n_steps % self.period == 0:                          # :358-362
            polyak(self.T, self.Q, self.tau)
        self.n_steps += 1
        self.last = dict(grads=dict(policy=S["gp"], target_policy=S["gtp"], qf=S["gq"]),
                         q_loss=S["q_loss"], std_loss=S["std_loss"], q_preds=S["q_preds"],
                         std_preds=S["std_preds"], q_target=S["q_target"],
                         std_target=S["std_target"], upper_bound=S["ub"], target_head=S["tpf"])
        return self.last


class ParticleUBOracle(GaussianOACOracle):
    """ParticleTrainer (trainer/particle_trainer.py, the p-oac recipes) with
    share_layers=True and the deterministic policy: critic Q with K particle
    outputs, sorted-particle TD targets (counts, std_soft_update,
    rescale_targets_around_mean) with the loss averaged over particles, the
    policy maximising sorted particle ``delta_index``, the target policy the
    particle mean.  Same phase split as GaussianOACOracle."""

    def __init__(self, params, obs_dim, act_dim, K, delta_index, q_min=0.0, q_max=100.0,
                 discount=0.99, reward_scale=1.0, policy_lr=1e-3, qf_lr=1e-3, tau=5e-3,
                 target_update_period=1, std_soft_update_prob=None, mean_update=False,
                 rescale=False, train_bias=True, next_policy=None, dtype=torch.float32):
        super().__init__(params, obs_dim, act_dim, q_min=q_min, q_max=q_max, discount=discount,
                         reward_scale=reward_scale, policy_lr=policy_lr, qf_lr=qf_lr, tau=tau,
                         target_update_period=target_update_period,
                         std_soft_update_prob=std_soft_update_prob, mean_update=mean_update,
                         train_bias=train_bias, next_policy=next_policy, dtype=dtype)
        self.K, self.delta_index = K, delta_index
        self.spread = (q_max - q_min) if rescale else None

    def phase0(self, batch):
        dt = self.dtype
        S = self.S = {}
        obs = S["obs"] = _t(batch["observations"], dt)
        act = _t(batch["actions"], dt)
        rew = _t(batch["rewards"], dt)
        term = _t(batch["terminals"], dt)
        nobs = _t(batch["next_observations"], dt)
        B = S["B"] = obs.shape[0]
        c = S["c"] = q_forward(obs, act, self.Q)                     # :190-195
        qs = c["q"].t()                                              # [K, B]
        sorted_qs, qs_idx = torch.sort(qs, dim=0)                    # :196
        pf2 = policy_forward(nobs, self._next_policy(), None, deterministic=True)   # :197-207
        tq = q_forward(nobs, pf2["a"], self.T)["q"].t()              # :211-214
        tq_sorted, _ = torch.sort(tq, dim=0)                         # :215
        y = self.reward_scale * rew.t() + (1. - term.t()) * self.discount * tq_sorted   # :219-220
        if self.soft is not None:                                    # :222-231
            cur_mean = torch.mean(sorted_qs, dim=0)
            nxt_mean = torch.mean(y, dim=0)
            y = self.soft * y + (1 - self.soft) * (sorted_qs - cur_mean + nxt_mean)
        if batch.get("counts") is not None:                          # :233-238
            cnt = _t(batch["counts"], dt).reshape(1, B)
            factor = (cnt == 0).to(dt)
            y = y * factor + (1 - factor) * (sorted_qs - torch.mean(sorted_qs, dim=0)
                                             + torch.mean(y, dim=0))
        if self.spread is not None:                                  # :254-262
            q_range = y[-1] - y[0]
            factor = torch.ones_like(q_range)
            factor[q_range > self.spread] = 0
            q_mean = torch.mean(y, dim=0)
            y = factor * y + (1 - factor) * ((y - q_mean) * (self.spread / (q_range + 1e-6))
                                             + q_mean)
        losses = ((sorted_qs - y) ** 2).mean(dim=1)                  # :264-268
        d_sorted = 2.0 * (sorted_qs - y) / B / self.K                # qf_loss /= K, :269
        S["dq"] = torch.zeros_like(qs).scatter_(0, qs_idx, d_sorted).t()
        S.update(sorted_qs=sorted_qs, y=y, tq=tq, qf_losses=losses, qf_loss=losses.sum() / self.K)
        S["pf"] = policy_forward(obs, self.P, None, deterministic=True)     # :309-311
        S["tpf"] = policy_forward(obs, self.TP, None, deterministic=True)   # :335-337

    def phase1(self, world=1):
        S = self.S
        S["gq"] = q_param_grads(S["c"], S["dq"], self.Q)
        if not self.train_bias:
            S["gq"]["last_fc.bias"] = torch.zeros_like(S["gq"]["last_fc.bias"])
        self.crit_flat = self._flat(S["gq"], list(self.Q))

    def phase2(self, world=1):
        S = self.S
        B, obs = S["B"], S["obs"]
        gq = self._unflat(self.crit_flat, self.Q, list(self.Q))
        self.opt_q.step({k: v / world for k, v in gq.items()})     # :270-272
        pf, tpf = S["pf"], S["tpf"]
        cn = q_forward(obs, pf["a"], self.Q)                         # :317 (post-step Q)
        pq = cn["q"].t()
        sq, sidx = torch.sort(pq, dim=0)                             # :322
        S["ub"] = sq[self.delta_index]                               # :323
        g0 = -torch.ones_like(S["ub"]) / B
        gsel = torch.zeros_like(pq).scatter_(0, sidx[self.delta_index:self.delta_index + 1],
                                             g0[None]).t()
        da = q_input_grad(cn, gsel, self.Q)[:, self.Do:]
        S["gp"] = det_policy_backward(pf, self.P, da)
        ct = q_forward(obs, tpf["a"], self.Q)                        # :339
        gt = (g0 / self.K)[:, None].expand(B, self.K)                # mean over particles :343
        dat = q_input_grad(ct, gt, self.Q)[:, self.Do:]
        S["gtp"] = det_policy_backward(tpf, self.TP, dat)
        self.pol_flat = torch.cat([self._flat(S["gp"], list(self.P)),
                                   self._flat(S["gtp"], list(self.TP))])

    def phase3(self, world=1):
        S = self.S
        n = self._flat(S["gp"], list(self.P)).numel()
        gp = self._unflat(self.pol_flat[:n], self.P, list(self.P))
        gtp = self._unflat(self.pol_flat[n:], self.TP, list(self.TP))
        self.opt_p.step({k: v / world for k, v in gp.items()})      # :329-330
        self.opt_tp.step({k: v / world for k, v in gtp.items()})    # :345-347
        if self.n_steps % self.period == 0:                          # :352-357
            polyak(self.T, self.Q, self.tau)
        self.n_steps += 1
        self.last = dict(grads=dict(policy=S["gp"], target_policy=S["gtp"], qf=S["gq"]),
                         qf_losses=S["qf_losses"], qf_loss=S["qf_loss"],
                         sorted_qs=S["sorted_qs"], y=S["y"], tq=S["tq"], upper_bound=S["ub"],
                         target_head=S["tpf"])
        return self.last


# ------------------------------------------------------- OAC exploration
def oac_exploration_action(ob_np, P, Q1, Q2, beta_UB, delta, eps_discard, eps,
                           dtype=torch.float32):
    """get_optimistic_exploration_action_stochastic (optimistic_exploration.py:14-109),
    trainer=None, two critics.  Returns (action, mu_E, std, grad)."""
    assert np.ndim(ob_np) == 1
    ob = _t(np.asarray(ob_np), dtype)[None]                   # from_numpy(...).float() :22
    pf = policy_forward(ob, P, _t(eps_discard, dtype)[None])  # :27 (draw discarded)
    mu_T, std = pf["mean"][0], pf["std"][0]
    a = torch.tanh(mu_T)                                       # :34
    c1 = q_forward(ob, a[None], Q1)                            # :41-44
    c2 = q_forward(ob, a[None], Q2)
    d = c1["q"] - c2["q"]
    sgn = torch.sign(d)
    w1 = 0.5 + (beta_UB / 2.0) * sgn                           # dQ_UB/dQ1 (:45-46,60)
    w2 = 0.5 - (beta_UB / 2.0) * sgn
    Do = ob.shape[1]
    ga = q_input_grad(c1, w1, Q1)[0, Do:] + q_input_grad(c2, w2, Q2)[0, Do:]
    grad = ga * (1 - a * a)                                    # tanh backward, :64
    Sigma = torch.pow(std, 2)                                  # :71
    denom = torch.sqrt(torch.sum(torch.mul(torch.pow(grad, 2), Sigma))) + 10e-6   # :76-80
    mu_C = math.sqrt(2.0 * delta) * torch.mul(Sigma, grad) / denom                # :83
    mu_E = mu_T + mu_C                                         # :87
    action = torch.tanh(_t(eps, dtype) * std + mu_E)           # TanhNormal(mu_E,std).sample() :92-94
    return dict(action=action, mu_E=mu_E, std=std, grad=grad, mu_T=mu_T)


def oac_exploration_action_shared(ob_np, P, Q, beta_UB, delta, eps_discard, eps,
                                  dtype=torch.float32, ub_index=None):
    """The same action with ONE shared-layer critic of K heads (share_layers=True,
    qfs = [qf]): qfs[1] raises, so the except branch of
    optimistic_exploration.py:47-56 takes mu_Q = mean_k Q_k, sigma_Q = std_k Q_k
    (unbiased), Q_UB = mu_Q + beta_UB sigma_Q;
    dQ_UB/dQ_k = 1/K + beta_UB (Q_k - mu_Q) / ((K-1) sigma_Q).

    ub_index (--trainer_UB with particle_trainer_oac.ParticleTrainer,
    optimistic_exploration.py:38-39 -> predict, particle_trainer_oac.py:147-167):
    Q_UB = sort_k(Q)[ub_index] (the trainer's delta_index), so the seed is 1 on
    the head sorted there (ties: the lower head index first) and 0 elsewhere."""
    assert np.ndim(ob_np) == 1
    ob = _t(np.asarray(ob_np), dtype)[None]
    pf = policy_forward(ob, P, _t(eps_discard, dtype)[None])
    mu_T, std = pf["mean"][0], pf["std"][0]
    a = torch.tanh(mu_T)
    c = q_forward(ob, a[None], Q)
    q = c["q"][0]                                              # [K]
    K = q.shape[0]
    if ub_index is None:
        mu = q.mean()
        sd = q.std()                                           # unbiased, like torch.std
        w = 1.0 / K + beta_UB * (q - mu) / ((K - 1) * sd)
    else:
        order = sorted(range(K), key=lambda k: (float(q[k]), k))
        w = torch.zeros_like(q)
        w[order[ub_index]] = 1.0
    Do = ob.shape[1]
    ga = q_input_grad(c, w[None], Q)[0, Do:]
    grad = ga * (1 - a * a)
    Sigma = torch.pow(std, 2)
    denom = torch.sqrt(torch.sum(torch.mul(torch.pow(grad, 2), Sigma))) + 10e-6
    mu_C = math.sqrt(2.0 * delta) * torch.mul(Sigma, grad) / denom
    mu_E = mu_T + mu_C
    action = torch.tanh(_t(eps, dtype) * std + mu_E)
    return dict(action=action, mu_E=mu_E, std=std, grad=grad, mu_T=mu_T)
