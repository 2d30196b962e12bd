"""Network producers with the reference's shapes and initialisation
(main.py:44-106 get_policy_producer / get_q_producer; networks.py:42-60 Mlp
init with ptu.fanin_init, utils/pytorch_util.py:17-26).

The trainers only read ``state_dict()`` from what a producer returns, so the
reference's own producers (returning its TanhGaussianPolicy / FlattenMlp)
plug in unchanged; these are for callers that do not have the reference
package (bench, smoke, tests).
"""
import numpy as np
import torch
from torch import nn


class InitMlp(nn.Module):
    """Parameter container with the reference's names and init:
    hidden W ~ U(+-1/sqrt(size[0])) (size[0] = out_features, rlkit's fanin_init
    quirk), hidden b = 0.1, last layer U(+-init_w)."""

    def __init__(self, in_dim, hidden_sizes, out_dim, init_w, log_std_head=False, bias=None,
                 device=None):
        super().__init__()
        d = in_dim
        for i, h in enumerate(hidden_sizes):
            fc = nn.Linear(d, h, device=device)
            bound = 1.0 / np.sqrt(fc.weight.size(0))
            with torch.no_grad():
                fc.weight.uniform_(-bound, bound)
                fc.bias.fill_(0.1)
            setattr(self, f"fc{i}", fc)
            d = h
        self.last_fc = nn.Linear(d, out_dim, device=device)
        with torch.no_grad():
            self.last_fc.weight.uniform_(-init_w, init_w)
            if bias is None:
                self.last_fc.bias.uniform_(-init_w, init_w)
            else:
                self.last_fc.bias.copy_(torch.as_tensor(np.asarray(bias, np.float32).reshape(out_dim)))
        if log_std_head:
            self.last_fc_log_std = nn.Linear(d, out_dim, device=device)
            with torch.no_grad():
                self.last_fc_log_std.weight.uniform_(-init_w, init_w)
                self.last_fc_log_std.bias.uniform_(-init_w, init_w)


def get_policy_producer(obs_dim, action_dim, hidden_sizes, device=None):
    def policy_producer(**kwargs):
        return InitMlp(obs_dim, hidden_sizes, action_dim, 1e-3, log_std_head=True, device=device)
    return policy_producer


def get_q_producer(obs_dim, action_dim, hidden_sizes, output_size=1, device=None):
    def q_producer(bias=None, positive=False, train_bias=True):
        return InitMlp(obs_dim + action_dim, hidden_sizes, output_size, 3e-3, bias=bias,
                       device=device)
    return q_producer
