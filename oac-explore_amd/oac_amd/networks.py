"""Arena-backed twins of the reference's networks.

``ArenaFlattenMlp`` / ``ArenaTanhGaussianPolicy`` are ``nn.Module``s whose
parameters are views into the trainer's flat HBM parameter arena (the buffers
the HIP kernels update in place).  They keep the reference's parameter names
and registration order (``fc0, fc1, ..., last_fc[, last_fc_log_std]`` --
/root/reference/networks.py:42-53, trainer/policies.py:241-243), so
``state_dict()`` / ``load_state_dict()`` / snapshots are interchangeable with
the reference's modules.

Their ``forward`` is the plain torch expression of the same math; it exists
for the callers outside the gradient-step hot path (evaluation rollouts via
``MakeDeterministic``, ``policy.get_action``).  The hot path itself -- the
gradient step and the optimistic exploration action -- runs in liboac_amd.
"""
import numpy as np
import torch
from torch import nn
import torch.nn.functional as F

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

    def forward(self, *inputs, **kwargs):
        h = torch.cat(inputs, dim=1)
        for fc in self.fcs:
            h = F.relu(fc(h))
        out = self.last_fc(h)
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
        self.oac_trainer = None  # set by the owning trainer (exploration handle)

    def forward(self, obs, reparameterize=True, deterministic=False, return_log_prob=False):
        h = obs
        for fc in self.fcs:
            h = F.relu(fc(h))
        mean = self.last_fc(h)
        log_std = torch.clamp(self.last_fc_log_std(h), LOG_SIG_MIN, LOG_SIG_MAX)
        std = torch.exp(log_std)
        log_prob = None
        if deterministic:
            action = torch.tanh(mean)
            pre_tanh = mean
        else:
            z = mean + std * torch.randn_like(mean)
            action = torch.tanh(z)
            pre_tanh = z
            if return_log_prob:
                lp = (-((z - mean) ** 2) / (2 * std ** 2) - torch.log(std)
                      - np.log(np.sqrt(2 * np.pi)) - torch.log(1 - action * action + 1e-6))
                log_prob = lp.sum(dim=-1, keepdim=True)
        if log_prob is None:
            log_prob = torch.zeros_like(action)
            pre_tanh = mean
        return action, mean, log_std, log_prob, std, pre_tanh

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
