"""Arena-backed twins of the reference's networks.

``ArenaFlattenMlp`` / ``ArenaTanhGaussianPolicy`` are ``nn.Module``s whose
parameters are views into the trainer's flat HBM parameter arena (the buffers
the HIP kernels update in place).  They keep the reference's parameter names
and registration order (``fc0, fc1, ..., last_fc[, last_fc_log_std]`` --
/root/reference/networks.py:42-53, trainer/policies.py:241-243), so
``state_dict()`` / ``load_state_dict()`` / snapshots are interchangeable with
the reference's modules.

Their ``forward`` (evaluation rollouts via ``MakeDeterministic``,
``policy.get_action``, ``trainer.predict``, user code) runs on liboac_amd's
row-wise network kernels (csrc/mlp_eval.hip); the critic forward is
differentiable w.r.t. its inputs (the kernel also returns d q / d [obs, act],
which the reference's exploration takes the gradient of:
optimistic_exploration.py:39, 64).  The gradient step and the optimistic
exploration action themselves run in liboac_amd's step / exploration plans.
"""
import ctypes

import numpy as np
import torch
from torch import nn
import torch.nn.functional as F

from . import _lib

LOG_SIG_MAX = 2
LOG_SIG_MIN = -20


class _ArenaLinear(nn.Module):
    def __init__(self, weight, bias):
        super().__init__()
        self.weight = nn.Parameter(weight, requires_grad=False)
        self.bias = nn.Parameter(bias, requires_grad=False)
        self.out_features, self.in_features = weight.shape

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


def _view(arena, off, *shape):
    n = int(np.prod(shape))
    return arena[off:off + n].view(*shape)


def _as_input(x, device):
    t = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))
    return t.to(device=device, dtype=torch.float32)


def _offsets(*offs):
    return (ctypes.c_int64 * 6)(*[int(o) for o in offs])


def critic_forward(mods, obs, act, need_jac):
    """q [N, len(mods) * Q] (and d q / d [obs | act] [N, len(mods) * Q, Do + Da])
    of one or two arena critics with the same layout (oac_critic_eval)."""
    m0 = mods[0]
    N, Do = obs.shape
    Da = act.shape[1] if act is not None else 0
    n, Q = len(mods), m0.output_size
    q = torch.empty(N, n * Q, dtype=torch.float32, device=obs.device)
    jac = torch.empty(N, n * Q, Do + Da, dtype=torch.float32, device=obs.device) if need_jac else None
    nets = (ctypes.c_void_p * 2)(*[m.arena.data_ptr() + 4 * m.base for m in mods] + [None] * (2 - n))
    _lib.check(_lib.lib().oac_critic_eval(
        nets, n, m0._offs, Do, Da, m0.hidden, Q, _lib.ptr(obs), Do,
        _lib.ptr(act) if act is not None else None, Da, N, _lib.ptr(q), _lib.ptr(jac),
        _lib.stream_ptr(torch.cuda.current_stream(obs.device))))
    return q, jac


class _CriticFn(torch.autograd.Function):
    """q = critics(obs, act) with the input gradient from the kernel's Jacobian."""

    @staticmethod
    def forward(ctx, obs, act, mods):
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        q, jac = critic_forward(mods, obs, act, need)
        ctx.save_for_backward(jac if need else None)
        ctx.Do = obs.shape[1]
        return q

    @staticmethod
    def backward(ctx, gq):
        jac, = ctx.saved_tensors
        gx = torch.bmm(gq.unsqueeze(1), jac).squeeze(1)
        return gx[:, :ctx.Do], gx[:, ctx.Do:], None


def critics_apply(mods, obs, act):
    """[N, len(mods) * Q] outputs of arena critics (before any `positive` exp)."""
    dev = mods[0].arena.device
    obs, act = _as_input(obs, dev), _as_input(act, dev)
    one = obs.dim() == 1
    if one:
        obs, act = obs[None], act[None]
    obs, act = obs.contiguous(), act.contiguous()
    if torch.is_grad_enabled() and (obs.requires_grad or act.requires_grad):
        q = _CriticFn.apply(obs, act, mods)
    else:
        q = critic_forward(mods, obs, act, False)[0]
    return q[0] if one else q


class ArenaFlattenMlp(nn.Module):
    """FlattenMlp (networks.py:154-161): relu hidden layers, identity output,
    inputs concatenated along dim 1."""

    def __init__(self, arena, base, layout, obs_dim, act_dim, hidden, out_dim, positive=False):
        super().__init__()
        L = layout
        self.positive = positive   # exp of the output (all, or per column), networks.py:69-75
        din = obs_dim + act_dim
        self.input_size, self.output_size = din, out_dim
        self.fc0 = _ArenaLinear(_view(arena, base + L.q_fc0_w, hidden, din),
                                _view(arena, base + L.q_fc0_b, hidden))
        self.fc1 = _ArenaLinear(_view(arena, base + L.q_fc1_w, hidden, hidden),
                                _view(arena, base + L.q_fc1_b, hidden))
        self.last_fc = _ArenaLinear(_view(arena, base + L.q_last_w, out_dim, hidden),
                                    _view(arena, base + L.q_last_b, out_dim))
        self.fcs = [self.fc0, self.fc1]
        self.arena, self.base = arena, base
        self.hidden, self.obs_dim, self.act_dim = hidden, obs_dim, act_dim
        self._offs = _offsets(L.q_fc0_w, L.q_fc0_b, L.q_fc1_w, L.q_fc1_b, L.q_last_w, L.q_last_b)

    def forward(self, *inputs, **kwargs):
        if len(inputs) == 2:
            out = critics_apply([self], inputs[0], inputs[1])
        else:   # FlattenMlp concatenates whatever it is given along dim 1
            x = torch.cat([_as_input(i, self.arena.device) for i in inputs], dim=1)
            out = critics_apply([self], x[:, :self.obs_dim], x[:, self.obs_dim:])
        if isinstance(self.positive, (list, tuple)):
            out = torch.stack([torch.exp(out[:, i]) if v else out[:, i]
                               for i, v in enumerate(self.positive)], dim=1)
        elif self.positive:
            out = torch.exp(out)
        return out


class ArenaTanhGaussianPolicy(nn.Module):
    """TanhGaussianPolicy (trainer/policies.py:195-316) over the arena; the
    two heads are stored stacked so the kernels read them as one matrix."""

    def __init__(self, arena, base, layout, obs_dim, act_dim, hidden):
        super().__init__()
        L = layout
        Da = act_dim
        hw = _view(arena, base + L.pol_head_w, 2 * Da, hidden)
        hb = _view(arena, base + L.pol_head_b, 2 * Da)
        self.fc0 = _ArenaLinear(_view(arena, base + L.pol_fc0_w, hidden, obs_dim),
                                _view(arena, base + L.pol_fc0_b, hidden))
        self.fc1 = _ArenaLinear(_view(arena, base + L.pol_fc1_w, hidden, hidden),
                                _view(arena, base + L.pol_fc1_b, hidden))
        self.last_fc = _ArenaLinear(hw[:Da], hb[:Da])
        self.last_fc_log_std = _ArenaLinear(hw[Da:], hb[Da:])
        self.fcs = [self.fc0, self.fc1]
        self.obs_dim, self.action_dim = obs_dim, act_dim
        self.input_size, self.output_size = obs_dim, act_dim
        self.std = None
        self.arena, self.base = arena, base
        self.hidden = hidden
        self._offs = _offsets(L.pol_fc0_w, L.pol_fc0_b, L.pol_fc1_w, L.pol_fc1_b, L.pol_head_w,
                              L.pol_head_b)
        self.oac_trainer = None  # set by the owning trainer (exploration handle)

    def forward(self, obs, reparameterize=True, deterministic=False, return_log_prob=False):
        """policies.py:260-316 on oac_policy_eval: the same 6-tuple (a
        non-sampled call returns log_prob = zeros_like(action) and pre_tanh =
        mean, as the reference does).  The noise is a torch.normal draw, as in
        TanhNormal.rsample (policies.py:182-186)."""
        dev = self.arena.device
        obs = _as_input(obs, dev)
        if torch.is_grad_enabled() and obs.requires_grad:
            raise NotImplementedError("oac_amd policy forward: no gradient w.r.t. the observation "
                                      "(the gradient step runs in the trainer's plan)")
        one = obs.dim() == 1
        x = (obs[None] if one else obs).contiguous()
        N, Da = x.shape[0], self.action_dim
        e = lambda *sh: torch.empty(*sh, dtype=torch.float32, device=dev)
        action, mean, log_std, std, pre = e(N, Da), e(N, Da), e(N, Da), e(N, Da), e(N, Da)
        sample = not deterministic
        eps = torch.randn(N, Da, device=dev) if sample else None
        lp = e(N) if (sample and return_log_prob) else None
        _lib.check(_lib.lib().oac_policy_eval(
            ctypes.c_void_p(self.arena.data_ptr() + 4 * self.base), self._offs, self.obs_dim, Da,
            self.hidden, _lib.ptr(x), self.obs_dim, N, _lib.ptr(eps), _lib.ptr(action),
            _lib.ptr(mean), _lib.ptr(log_std), _lib.ptr(lp), _lib.ptr(std), _lib.ptr(pre),
            _lib.stream_ptr(torch.cuda.current_stream(dev))))
        if lp is not None:
            log_prob = lp.view(N, 1)
        else:
            log_prob = torch.zeros_like(action)
            pre = mean
        out = (action, mean, log_std, log_prob, std, pre)
        return tuple(t[0] for t in out) if one else out

    def get_action(self, obs_np, deterministic=False):
        actions = self.get_actions(obs_np[None], deterministic=deterministic)
        return actions[0, :], {}

    @torch.no_grad()
    def get_actions(self, obs_np, deterministic=False):
        obs = torch.as_tensor(np.asarray(obs_np), dtype=torch.float32, device=self.arena.device)
        return self(obs, deterministic=deterministic)[0].cpu().numpy()

    def reset(self):
        pass


class MakeDeterministic(nn.Module):
    """Evaluation wrapper (trainer/policies.py:486-513)."""

    def __init__(self, stochastic_policy):
        super().__init__()
        self.stochastic_policy = stochastic_policy

    def get_action(self, observation, deterministic=True):
        return self.stochastic_policy.get_action(observation, deterministic=True)

    def get_actions(self, observations):
        return self.stochastic_policy.get_actions(observations, deterministic=True)

    def forward(self, *args, **kwargs):
        kwargs["deterministic"] = True
        return self.stochastic_policy.forward(*args, **kwargs)

    def reset(self):
        pass
