"""Row-wise network evaluation on the HIP kernels (csrc/mlp_eval.hip): the
arena modules' forward, SACTrainer.predict and ParticleTrainer.predict
(trainer/trainer.py:105-123, particle_trainer_oac.py:147-167) against the CPU
oracle, including the gradient of Q_UB w.r.t. the action that the
reference's exploration takes (optimistic_exploration.py:33-64)."""
import numpy as np
import pytest
import torch

import parity
from fixtures_lib import sac_params
from gpu_helpers import Space, producers, sac_trainer_for
from oracle import sac_oracle as so

pytestmark = pytest.mark.gpu

Do, Da, H = 376, 17, 256
META = dict(obs_dim=Do, act_dim=Da, hidden=[H, H], discount=0.99, reward_scale=1.0, lr=3e-4,
            tau=5e-3, auto_alpha=True, log_alpha0=0.0, seed=5, pi_init_w=0.3, q_init_w=0.3)


def _params():
    return sac_params(Do, Da, [H, H], META["seed"], pi_init_w=META["pi_init_w"],
                      q_init_w=META["q_init_w"])


def _oracle_q(p, obs, act):
    P = so.to_torch_params(p, torch.float64)
    return so.q_forward(torch.as_tensor(obs, dtype=torch.float64),
                        torch.as_tensor(act, dtype=torch.float64), P)["q"]


@pytest.mark.parametrize("n", [1, 7, 64])
def test_sac_predict_and_its_action_gradient_match_the_oracle(n):
    prm = _params()
    tr = sac_trainer_for(META, params=prm)
    rs = np.random.RandomState(n)
    obs = rs.standard_normal((n, Do)).astype(np.float32)
    pre = rs.standard_normal((n, Da)).astype(np.float32)
    beta = 4.66
    # ours: the reference's exploration recipe against trainer.predict
    mu_t = torch.tensor(pre, device="cuda:0", requires_grad=True)
    q_ub = tr.predict(torch.tensor(obs, device="cuda:0"), torch.tanh(mu_t), beta_UB=beta)
    g, = torch.autograd.grad(q_ub.sum(), mu_t)
    # oracle: float64 autograd through the same formula
    mo = torch.tensor(pre, dtype=torch.float64, requires_grad=True)
    a = torch.tanh(mo)
    q1, q2 = _oracle_q(prm["qf1"], obs, a), _oracle_q(prm["qf2"], obs, a)
    ub = (q1 + q2) / 2 + beta * torch.abs(q1 - q2) / 2
    go, = torch.autograd.grad(ub.sum(), mo)
    assert parity.rel_err(q_ub.detach().cpu().numpy(), ub.detach().numpy()) < 1e-5
    assert parity.rel_err(g.cpu().numpy(), go.numpy()) < 1e-5
    mu, sig = tr.predict(obs, np.tanh(pre), both_values=True)
    assert parity.rel_err(mu.cpu().numpy(), ((q1 + q2) / 2).detach().numpy()) < 1e-5
    assert parity.rel_err(sig.cpu().numpy(), (torch.abs(q1 - q2) / 2).detach().numpy()) < 1e-5
    if n == 1:   # 1-D inputs are unsqueezed (trainer.py:109-110)
        one = tr.predict(obs[0], np.tanh(pre[0]), beta_UB=beta)
        assert one.shape == (1, 1)


def test_critic_module_forward_and_input_gradient():
    prm = _params()
    tr = sac_trainer_for(META, params=prm)
    rs = np.random.RandomState(3)
    obs = torch.tensor(rs.standard_normal((33, Do)), dtype=torch.float32, device="cuda:0",
                       requires_grad=True)
    act = torch.tensor(rs.uniform(-1, 1, (33, Da)), dtype=torch.float32, device="cuda:0",
                       requires_grad=True)
    q = tr.qf2(obs, act)
    go, ga = torch.autograd.grad((q * q).sum(), (obs, act))
    o64 = obs.detach().cpu().double().requires_grad_()
    a64 = act.detach().cpu().double().requires_grad_()
    qr = so.q_forward(o64, a64, so.to_torch_params(prm["qf2"], torch.float64))["q"]
    gro, gra = torch.autograd.grad((qr * qr).sum(), (o64, a64))
    assert parity.rel_err(q.detach().cpu().numpy(), qr.detach().numpy()) < 1e-5
    assert parity.rel_err(go.cpu().numpy(), gro.numpy()) < 1e-5
    assert parity.rel_err(ga.cpu().numpy(), gra.numpy()) < 1e-5


def test_policy_module_forward_matches_the_oracle():
    # the reference's policy head init (init_w 1e-3, policies.py:220): no tanh
    # saturation, where log(1 - a^2 + 1e-6) would amplify fp32 rounding
    meta = dict(META, pi_init_w=1e-3)
    prm = sac_params(Do, Da, [H, H], META["seed"], pi_init_w=1e-3, q_init_w=0.3)
    tr = sac_trainer_for(meta, params=prm)
    rs = np.random.RandomState(4)
    obs = rs.standard_normal((40, Do)).astype(np.float32)
    P = so.to_torch_params(prm["policy"], torch.float64)
    # deterministic (MakeDeterministic / eval rollouts): tanh(mean), log_prob zeros
    a, mean, log_std, lp, std, pre = tr.policy(torch.tensor(obs), deterministic=True)
    ref = so.policy_forward(torch.tensor(obs, dtype=torch.float64), P,
                            torch.zeros(40, Da, dtype=torch.float64), deterministic=True)
    assert parity.rel_err(mean.cpu().numpy(), ref["mean"].numpy()) < 1e-5
    assert parity.rel_err(log_std.cpu().numpy(), ref["log_std"].numpy()) < 1e-5
    assert parity.rel_err(a.cpu().numpy(), np.tanh(ref["mean"].numpy())) < 1e-5
    assert torch.equal(pre, mean) and lp.shape == a.shape and not lp.any()
    # stochastic with log-prob: the noise the kernel used is (pre_tanh - mean) / std
    torch.manual_seed(0)
    a, mean, log_std, lp, std, z = tr.policy(torch.tensor(obs), return_log_prob=True)
    eps = ((z - mean) / std).double().cpu()
    ref = so.policy_forward(torch.tensor(obs, dtype=torch.float64), P, eps)
    assert parity.rel_err(a.cpu().numpy(), ref["a"].numpy()) < 1e-5
    assert parity.rel_err(lp.cpu().numpy(), ref["logp"].numpy()) < 1e-5
    assert lp.shape == (40, 1)
    # get_action (rollouts): one observation in, one action out
    act, info = tr.policy.get_action(obs[0])
    assert act.shape == (Da,) and info == {} and np.all(np.abs(act) <= 1)


def test_particle_predict_and_gradient_match_the_oracle():
    from oac_amd import ParticleTrainerOAC
    K = 10
    prm = sac_params(111, 8, [256, 256], 6, q_out=K, pi_init_w=0.3, q_init_w=0.3,
                     q_last_bias=np.linspace(0.0, 50.0, K))
    pp, qp = producers(prm, q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                    "target_qf1"))
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(8), discount=0.99,
                            policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3, delta=0.95,
                            use_automatic_entropy_tuning=True, deterministic=False, q_min=0.0,
                            q_max=50.0, share_layers=True)
    rs = np.random.RandomState(8)
    obs = rs.standard_normal((5, 111)).astype(np.float32)
    pre = rs.standard_normal((5, 8)).astype(np.float32)
    mu_t = torch.tensor(pre, device="cuda:0", requires_grad=True)
    out = tr.predict(torch.tensor(obs, device="cuda:0"), torch.tanh(mu_t))
    g, = torch.autograd.grad(out.sum(), mu_t)
    mo = torch.tensor(pre, dtype=torch.float64, requires_grad=True)
    qs = _oracle_q(prm["qf1"], obs, torch.tanh(mo)).t().unsqueeze(-1)
    ref = torch.sort(qs, dim=0)[0][tr.delta_index]
    go, = torch.autograd.grad(ref.sum(), mo)
    assert out.shape == (5, 1)
    assert parity.rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) < 1e-5
    assert parity.rel_err(g.cpu().numpy(), go.numpy()) < 1e-5
    mean = tr.predict(obs, np.tanh(pre), upper_bound=False)
    assert parity.rel_err(mean.cpu().numpy(), torch.mean(qs, 0).detach().numpy()) < 1e-5
