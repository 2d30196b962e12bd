"""Shared deterministic inputs for the parity fixtures (test infrastructure).

Both the golden generator (which runs the reference in this container) and the
GPU parity tests build their parameters and transitions from these functions,
so the reference and the HIP path start from bit-identical fp32 state.

Parameter names follow the reference's ``state_dict`` keys:
``Mlp`` registers ``fc0, fc1, ..., last_fc`` (/root/reference/networks.py:42-53)
and ``TanhGaussianPolicy`` adds ``last_fc_log_std``
(/root/reference/trainer/policies.py:241-243).  The distributions follow the
reference's init (networks.py:45-53, utils/pytorch_util.py:17-26): hidden
weights U(+-1/sqrt(size[0])) with size[0] = out_features, hidden bias 0.1,
last layer U(+-init_w) -- but drawn from numpy so the fixture is seedable
independently of torch's generator.
"""
import numpy as np


def mlp_params(rs, in_dim, hidden, out_dim, init_w, log_std_head=False,
               last_bias=None):
    p = {}
    d = in_dim
    for i, h in enumerate(hidden):
        bound = 1.0 / np.sqrt(h)  # fan_in = size[0] = out_features (rlkit quirk)
        p[f"fc{i}.weight"] = rs.uniform(-bound, bound, (h, d)).astype(np.float32)
        p[f"fc{i}.bias"] = np.full((h,), 0.1, np.float32)
        d = h
    p["last_fc.weight"] = rs.uniform(-init_w, init_w, (out_dim, d)).astype(np.float32)
    if last_bias is None:
        p["last_fc.bias"] = rs.uniform(-init_w, init_w, (out_dim,)).astype(np.float32)
    else:
        p["last_fc.bias"] = np.asarray(last_bias, np.float32).reshape(out_dim)
    if log_std_head:
        p["last_fc_log_std.weight"] = rs.uniform(-init_w, init_w, (out_dim, d)).astype(np.float32)
        p["last_fc_log_std.bias"] = rs.uniform(-init_w, init_w, (out_dim,)).astype(np.float32)
    return p


def sac_params(obs_dim, act_dim, hidden, seed, q_out=1, pi_init_w=1e-3,
               q_init_w=3e-3, q_last_bias=None):
    """policy, qf1, qf2, target_qf1, target_qf2 parameter dicts (fp32)."""
    rs = np.random.RandomState(seed)
    pol = mlp_params(rs, obs_dim, hidden, act_dim, pi_init_w, log_std_head=True)
    qf1 = mlp_params(rs, obs_dim + act_dim, hidden, q_out, q_init_w, last_bias=q_last_bias)
    qf2 = mlp_params(rs, obs_dim + act_dim, hidden, q_out, q_init_w, last_bias=q_last_bias)
    tq1 = mlp_params(rs, obs_dim + act_dim, hidden, q_out, q_init_w, last_bias=q_last_bias)
    tq2 = mlp_params(rs, obs_dim + act_dim, hidden, q_out, q_init_w, last_bias=q_last_bias)
    return dict(policy=pol, qf1=qf1, qf2=qf2, target_qf1=tq1, target_qf2=tq2)


def goac_params(obs_dim, act_dim, hidden, seed, q_min, q_max, pi_init_w=1e-3, q_init_w=3e-3):
    """g-oac (GaussianTrainer, share_layers): policy, target_policy, qf1
    (outputs Q | log std, last bias [mean, log std] of the uniform prior on
    [q_min, q_max], gaussian_trainer.py:70-92) and target_qf1 (fp32)."""
    bias = [(q_max + q_min) / 2, np.log((q_max - q_min) / np.sqrt(12))]
    d = sac_params(obs_dim, act_dim, hidden, seed, q_out=2, pi_init_w=pi_init_w,
                   q_init_w=q_init_w, q_last_bias=bias)
    rs = np.random.RandomState(seed + 1)
    tp = mlp_params(rs, obs_dim, hidden, act_dim, pi_init_w, log_std_head=True)
    return dict(policy=d["policy"], target_policy=tp, qf1=d["qf1"], target_qf1=d["target_qf1"])


def ptrain_params(obs_dim, act_dim, hidden, seed, K, q_min, q_max, pi_init_w=1e-3,
                  q_init_w=3e-3):
    """p-oac ParticleTrainer (particle_trainer.py, share_layers): policy,
    target_policy, qf1 (K particles, last bias linspace(q_min, q_max, K)) and
    target_qf1 = qf1 (the constructor copies it, soft_update tau=1, :100-102)."""
    d = sac_params(obs_dim, act_dim, hidden, seed, q_out=K, pi_init_w=pi_init_w,
                   q_init_w=q_init_w, q_last_bias=np.linspace(q_min, q_max, K))
    rs = np.random.RandomState(seed + 1)
    tp = mlp_params(rs, obs_dim, hidden, act_dim, pi_init_w, log_std_head=True)
    return dict(policy=d["policy"], target_policy=tp, qf1=d["qf1"],
                target_qf1={k: v.copy() for k, v in d["qf1"].items()})


def mid_state(params, groups, t, seed, g_scale=1e-2):
    """A mid-training optimiser state (test infrastructure): torch-Adam moments
    after ``t`` steps for every tensor of ``params[group]`` (group in
    ``groups``), plus log-alpha and its moments.  exp_avg ~ N(0, g_scale),
    exp_avg_sq = exp_avg^2 + Exp(g_scale^2) (so sqrt(v) >= |m|, as a real run
    keeps it).  The mid-state goldens (make_golden.py gen_sac_mid /
    gen_poac_mid) run ONE reference step from this state, so steps past the
    first -- bias corrections at t > 1, non-zero moments, log-alpha away from
    its init -- are pinned against the reference at 1e-5 without storing a
    trajectory's state."""
    rs = np.random.RandomState(seed)
    out = {}
    for g in groups:
        out[g] = {}
        for k, v in params[g].items():
            m = rs.normal(0.0, g_scale, v.shape).astype(np.float32)
            vv = (m.astype(np.float64) ** 2 + rs.exponential(g_scale ** 2, v.shape)).astype(np.float32)
            out[g][k] = (m, vv)
    out["log_alpha"] = np.float32(rs.uniform(-0.6, -0.2))
    am = np.float32(rs.normal(0.0, g_scale))
    out["alpha_adam"] = (am, np.float32(am * am + rs.exponential(g_scale ** 2)))
    out["t"] = int(t)
    return out


def synthetic_transitions(n, obs_dim, act_dim, seed=0, term_p=0.01):
    """BASELINE.md section 3 synthetic replay content (float64, like the
    reference's numpy store, replay_buffer.py:32-45)."""
    rs = np.random.RandomState(seed)
    obs = rs.standard_normal((n, obs_dim))
    act = rs.uniform(-1.0, 1.0, (n, act_dim))
    rew = rs.standard_normal((n, 1))
    term = (rs.uniform(0.0, 1.0, (n, 1)) < term_p).astype(np.uint8)
    nobs = rs.standard_normal((n, obs_dim))
    return dict(observations=obs, actions=act, rewards=rew, terminals=term,
                next_observations=nobs)


PARAM_ORDER_POLICY = ["fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias",
                      "last_fc.weight", "last_fc.bias",
                      "last_fc_log_std.weight", "last_fc_log_std.bias"]
PARAM_ORDER_Q = ["fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias",
                 "last_fc.weight", "last_fc.bias"]
