"""Generate the golden parity fixtures by running the REFERENCE itself.

Runs only in the build container (it imports the read-only reference from
/root/reference; nothing under tests/golden/*.npz contains reference code --
only inputs and the outputs the reference produced on them).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Harness shims (all on the harness side, the reference files are untouched):
  * ``gym`` / ``gym.spaces`` stub so ``replay_buffer.ReplayBuffer`` imports
    (it only needs ``Box``/``Discrete``/``Tuple`` for ``get_dim``,
    /root/reference/utils/env_utils.py:8-18);
  * ``Adam14``: torch-1.4 Adam semantics passed through the reference's own
    ``optimizer_class`` constructor argument (trainer/trainer.py:24,75-91).
    It updates through ``p.data`` exactly like torch 1.4 did, which is what
    lets ``policy_loss.backward()`` (trainer/trainer.py:209) run after the Q
    steps and see the post-step Q weights.
    It also records the gradient of every parameter at step() time;
  * ``Normal.sample`` is wrapped to record the standard-normal draw eps
    behind every sample (replayed from the saved RNG state and checked
    bit-for-bit against the reference's own output).
"""
import math
import os
import zlib
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # tests/
from fixtures_lib import (goac_params, mid_state, ptrain_params, sac_params, synthetic_transitions,  # noqa
                          PARAM_ORDER_POLICY, PARAM_ORDER_Q)

REF = "/root/reference"


# ----------------------------------------------------------------- gym stub
def _install_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            shape = shape if shape is not None else np.shape(low)
            self.low = np.broadcast_to(np.asarray(low, np.float32), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, np.float32), shape).copy()
            self.shape = tuple(shape)

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Tuple:
        def __init__(self, spaces_):
            self.spaces = spaces_

    class Env:
        pass

    spaces.Box, spaces.Discrete, spaces.Tuple = Box, Discrete, Tuple
    gym.spaces, gym.Env = spaces, Env
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces
    return Box


Box = _install_gym_stub()
sys.path.insert(0, REF)
import utils.pytorch_util as ptu  # noqa: E402

ptu.set_gpu_mode(False)
from networks import FlattenMlp  # noqa: E402
from trainer.policies import TanhGaussianPolicy  # noqa: E402
from trainer.trainer import SACTrainer  # noqa: E402
from trainer.particle_trainer_oac import ParticleTrainer as ParticleTrainerOAC  # noqa: E402
from trainer.gaussian_trainer import GaussianTrainer  # noqa: E402
from trainer.particle_trainer import ParticleTrainer  # noqa: E402
from replay_buffer import ReplayBuffer, ReplayBufferCount  # noqa: E402
import optimistic_exploration as oe  # noqa: E402


# ------------------------------------------------------ torch-1.4 Adam shim
class Adam14(torch.optim.Optimizer):
    """torch 1.4.0 ``optim.Adam.step`` semantics (p.data updates, no version bump)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.recorded = []

    def step(self, closure=None):
        rec = []
        with torch.no_grad():
            for group in self.param_groups:
                b1, b2 = group["betas"]
                for p in group["params"]:
                    if p.grad is None:
                        rec.append(None)
                        continue
                    g = p.grad.data
                    rec.append(g.detach().clone())
                    st = self.state[p]
                    if len(st) == 0:
                        st["step"] = 0
                        st["exp_avg"] = torch.zeros_like(p.data)
                        st["exp_avg_sq"] = torch.zeros_like(p.data)
                    m, v = st["exp_avg"], st["exp_avg_sq"]
                    st["step"] += 1
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    bc1 = 1 - b1 ** st["step"]
                    bc2 = 1 - b2 ** st["step"]
                    denom = (v.sqrt() / math.sqrt(bc2)).add_(group["eps"])
                    p.data.addcdiv_(m, denom, value=-(group["lr"] / bc1))
        self.recorded.append(rec)


# ------------------------------------------------------------ eps recorder
EPS_LOG = []
_orig_sample = torch.distributions.Normal.sample


def _recording_sample(self, sample_shape=torch.Size()):
    st = torch.get_rng_state()
    out = _orig_sample(self, sample_shape)
    after = torch.get_rng_state()
    torch.set_rng_state(st)
    shape = out.shape
    eps = torch.normal(torch.zeros(shape), torch.ones(shape))
    torch.set_rng_state(after)
    recon = eps * self.scale.expand(shape) + self.loc.expand(shape)
    assert torch.equal(recon, out), "eps replay does not reproduce Normal.sample"
    EPS_LOG.append(eps.numpy().copy())
    return out


torch.distributions.Normal.sample = _recording_sample


# ---------------------------------------------------------------- packing
SAMPLE_N = 512


def pack(out, key, arr, full):
    arr = np.array(arr, np.float32, copy=True)  # state_dict tensors alias live params
    if full or arr.size <= 2048:
        out[key] = arr
        return
    flat = arr.reshape(-1)
    rs = np.random.RandomState(zlib.crc32(key.encode()) % (2 ** 31))
    idx = np.sort(rs.choice(flat.size, SAMPLE_N, replace=False)).astype(np.int64)
    out[key + "#norm"] = np.array(np.linalg.norm(flat.astype(np.float64)))
    out[key + "#idx"] = idx
    out[key + "#val"] = flat[idx]
    out[key + "#shape"] = np.array(arr.shape, np.int64)


def load_sd(module, d):
    module.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in d.items()})


def _producers(obs_dim, act_dim, hidden, q_out=1):
    def policy_producer(**kw):
        return TanhGaussianPolicy(hidden_sizes=hidden, obs_dim=obs_dim, action_dim=act_dim)

    def q_producer(bias=None, positive=False, train_bias=True):
        return FlattenMlp(input_size=obs_dim + act_dim, output_size=q_out,
                          hidden_sizes=hidden, bias=bias, positive=positive,
                          train_bias=train_bias)
    return policy_producer, q_producer


def _fill_buffer(obs_dim, act_dim, n, seed=0):
    rb = ReplayBuffer(n, Box(-1, 1, (obs_dim,)), Box(-1, 1, (act_dim,)))
    tr = synthetic_transitions(n, obs_dim, act_dim, seed=seed)
    for i in range(n):
        rb.add_sample(tr["observations"][i], tr["actions"][i], tr["rewards"][i],
                      tr["next_observations"][i], tr["terminals"][i], env_info={})
    return rb, tr


def _record_batch(rb, B):
    st = np.random.get_state()
    batch = rb.random_batch(B)
    rs = np.random.RandomState()
    rs.set_state(st)
    idx = rs.randint(0, rb._size, B)
    assert np.array_equal(batch["observations"], rb._observations[idx])
    return batch, idx


# -------------------------------------------------------------- SAC runs
def gen_sac(name, obs_dim, act_dim, hidden, B, steps, n_replay, full, seed=7,
            pi_init_w=1e-3, q_init_w=3e-3, auto_alpha=True, log_alpha0=0.0,
            discount=0.99, reward_scale=1.0, tau=5e-3, lr=3e-4, idx_seed=1,
            eps_seed=2, full_s0=False, period=1):
    """full_s0: step 0's gradients and post-step parameters stored whole (not
    sampled) even at hidden 256, so the headline configs are checked
    element for element at 1e-5."""
    pp, qp = _producers(obs_dim, act_dim, hidden)
    torch.manual_seed(0)
    tr = SACTrainer(pp, qp, action_space=Box(-1, 1, (act_dim,)), discount=discount,
                    reward_scale=reward_scale, policy_lr=lr, qf_lr=lr,
                    optimizer_class=Adam14, soft_target_tau=tau, target_update_period=period,
                    use_automatic_entropy_tuning=auto_alpha)
    params = sac_params(obs_dim, act_dim, hidden, seed, pi_init_w=pi_init_w, q_init_w=q_init_w)
    load_sd(tr.policy, params["policy"])
    for k in ("qf1", "qf2", "target_qf1", "target_qf2"):
        load_sd(getattr(tr, k), params[k])
    if auto_alpha:
        tr.log_alpha.data.fill_(log_alpha0)
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    np.random.seed(idx_seed)
    torch.manual_seed(eps_seed)
    out = {}
    meta = dict(kind="sac", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, B=B, steps=steps,
                n_replay=n_replay, seed=seed, pi_init_w=pi_init_w, q_init_w=q_init_w,
                auto_alpha=auto_alpha, log_alpha0=log_alpha0, discount=discount,
                reward_scale=reward_scale, tau=tau, lr=lr, idx_seed=idx_seed,
                eps_seed=eps_seed, target_entropy=-float(act_dim), target_update_period=period)
    for s in range(steps):
        EPS_LOG.clear()
        batch, idx = _record_batch(rb, B)
        tr.end_epoch(s)  # force the eval statistics for this step
        tr.train(dict(batch))
        assert len(EPS_LOG) == 2
        out[f"s{s}/idx"] = idx.astype(np.int64)
        out[f"s{s}/eps1"] = EPS_LOG[0]
        out[f"s{s}/eps2"] = EPS_LOG[1]
        stats = tr.get_diagnostics()
        for k, v in stats.items():
            out[f"s{s}/stat/{k}"] = np.array(v, np.float64)
        groups = [("policy", tr.policy_optimizer, PARAM_ORDER_POLICY),
                  ("qf1", tr.qf1_optimizer, PARAM_ORDER_Q),
                  ("qf2", tr.qf2_optimizer, PARAM_ORDER_Q)]
        for gname, opt, order in groups:
            grads = opt.recorded[-1]
            for pname, g in zip(order, grads):
                pack(out, f"s{s}/grad/{gname}/{pname}", g.numpy(), full or (full_s0 and s == 0))
        if auto_alpha:
            out[f"s{s}/grad/log_alpha"] = tr.alpha_optimizer.recorded[-1][0].numpy()
            out[f"s{s}/post/log_alpha"] = tr.log_alpha.detach().numpy().copy()
        for gname in ("policy", "qf1", "qf2", "target_qf1", "target_qf2"):
            for pname, t in getattr(tr, gname).state_dict().items():
                pack(out, f"s{s}/post/{gname}/{pname}", t.numpy(), full or (full_s0 and s == 0))
        for gname, opt in (("policy", tr.policy_optimizer), ("qf1", tr.qf1_optimizer)):
            order = PARAM_ORDER_POLICY if gname == "policy" else PARAM_ORDER_Q
            for pname, p in zip(order, opt.param_groups[0]["params"]):
                st = opt.state[p]
                pack(out, f"s{s}/adam/{gname}/{pname}/exp_avg", st["exp_avg"].numpy(), full)
                pack(out, f"s{s}/adam/{gname}/{pname}/exp_avg_sq", st["exp_avg_sq"].numpy(), full)
    return meta, out


# ------------------------------------------------- mid-training-state runs
def _set_adam(opt, order, st, t):
    """torch-Adam state (Adam14's layout) of every parameter of ``opt``."""
    for pname, p in zip(order, opt.param_groups[0]["params"]):
        m, v = st[pname]
        opt.state[p] = dict(step=t, exp_avg=torch.from_numpy(m.copy()),
                            exp_avg_sq=torch.from_numpy(v.copy()))


def _set_alpha(tr, ms):
    tr.log_alpha.data.fill_(float(ms["log_alpha"]))
    am, av = ms["alpha_adam"]
    tr.alpha_optimizer.state[tr.log_alpha] = dict(
        step=ms["t"], exp_avg=torch.tensor([am]), exp_avg_sq=torch.tensor([av]))


def gen_sac_mid(name, obs_dim, act_dim, hidden, B, n_replay, t=7, seed=7, state_seed=31,
                lr=3e-4, tau=5e-3, idx_seed=3, eps_seed=4):
    """ONE reference SAC step from a mid-training state (fixtures_lib.mid_state:
    Adam moments after t steps, log-alpha off its init): gradients whole,
    post-step parameters / targets / Adam moments sampled."""
    pp, qp = _producers(obs_dim, act_dim, hidden)
    torch.manual_seed(0)
    tr = SACTrainer(pp, qp, action_space=Box(-1, 1, (act_dim,)), discount=0.99,
                    reward_scale=1.0, policy_lr=lr, qf_lr=lr, optimizer_class=Adam14,
                    soft_target_tau=tau, target_update_period=1,
                    use_automatic_entropy_tuning=True)
    params = sac_params(obs_dim, act_dim, hidden, seed)
    for k in ("policy", "qf1", "qf2", "target_qf1", "target_qf2"):
        load_sd(getattr(tr, k), params[k])
    ms = mid_state(params, ("policy", "qf1", "qf2"), t, state_seed)
    _set_adam(tr.policy_optimizer, PARAM_ORDER_POLICY, ms["policy"], t)
    _set_adam(tr.qf1_optimizer, PARAM_ORDER_Q, ms["qf1"], t)
    _set_adam(tr.qf2_optimizer, PARAM_ORDER_Q, ms["qf2"], t)
    _set_alpha(tr, ms)
    tr._n_train_steps_total = t
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    np.random.seed(idx_seed)
    torch.manual_seed(eps_seed)
    EPS_LOG.clear()
    batch, idx = _record_batch(rb, B)
    tr.end_epoch(0)
    tr.train(dict(batch))
    assert len(EPS_LOG) == 2
    out = {"s0/idx": idx.astype(np.int64), "s0/eps1": EPS_LOG[0], "s0/eps2": EPS_LOG[1]}
    for k, v in tr.get_diagnostics().items():
        out[f"s0/stat/{k}"] = np.array(v, np.float64)
    for gname, opt, order in (("policy", tr.policy_optimizer, PARAM_ORDER_POLICY),
                              ("qf1", tr.qf1_optimizer, PARAM_ORDER_Q),
                              ("qf2", tr.qf2_optimizer, PARAM_ORDER_Q)):
        for pname, g, p in zip(order, opt.recorded[-1], opt.param_groups[0]["params"]):
            pack(out, f"s0/grad/{gname}/{pname}", g.numpy(), True)
            st = opt.state[p]
            pack(out, f"s0/adam/{gname}/{pname}/exp_avg", st["exp_avg"].numpy(), False)
            pack(out, f"s0/adam/{gname}/{pname}/exp_avg_sq", st["exp_avg_sq"].numpy(), False)
    out["s0/grad/log_alpha"] = tr.alpha_optimizer.recorded[-1][0].numpy()
    out["s0/post/log_alpha"] = tr.log_alpha.detach().numpy().copy()
    for gname in ("policy", "qf1", "qf2", "target_qf1", "target_qf2"):
        for pname, tt in getattr(tr, gname).state_dict().items():
            pack(out, f"s0/post/{gname}/{pname}", tt.numpy(), False)
    meta = dict(kind="sac", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, B=B, steps=1,
                n_replay=n_replay, seed=seed, pi_init_w=1e-3, q_init_w=3e-3, auto_alpha=True,
                log_alpha0=float(ms["log_alpha"]), discount=0.99, reward_scale=1.0, tau=tau,
                lr=lr, idx_seed=idx_seed, eps_seed=eps_seed, target_entropy=-float(act_dim),
                target_update_period=1, mid_state=dict(t=t, seed=state_seed))
    return meta, out


def gen_poac_mid(name, obs_dim, act_dim, hidden, K, B, n_replay, t=7, seed=11, state_seed=37,
                 q_min=0.0, q_max=500.0, lr=3e-4, tau=5e-3, idx_seed=3, eps_seed=4):
    """ONE reference P-OAC step (particle_trainer_oac, share_layers) from a
    mid-training state; gradients whole, the rest sampled."""
    pp, qp = _producers(obs_dim, act_dim, hidden, q_out=K)
    torch.manual_seed(0)
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Box(-1, 1, (act_dim,)),
                            discount=0.99, reward_scale=1.0, delta=0.95, policy_lr=lr,
                            qf_lr=lr, optimizer_class=Adam14, soft_target_tau=tau,
                            target_update_period=1, use_automatic_entropy_tuning=True,
                            deterministic=False, q_min=q_min, q_max=q_max, share_layers=True)
    params = sac_params(obs_dim, act_dim, hidden, seed, q_out=K,
                        q_last_bias=np.linspace(q_min, q_max, K))
    load_sd(tr.policy, params["policy"])
    load_sd(tr.qfs[0], params["qf1"])
    load_sd(tr.tfs[0], params["target_qf1"])
    ms = mid_state(params, ("policy", "qf1"), t, state_seed)
    _set_adam(tr.policy_optimizer, PARAM_ORDER_POLICY, ms["policy"], t)
    _set_adam(tr.qf_optimizers[0], PARAM_ORDER_Q, ms["qf1"], t)
    _set_alpha(tr, ms)
    tr._n_train_steps_total = t
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    np.random.seed(idx_seed)
    torch.manual_seed(eps_seed)
    EPS_LOG.clear()
    batch, idx = _record_batch(rb, B)
    tr.end_epoch(0)
    tr.train(dict(batch))
    assert len(EPS_LOG) == 2
    out = {"s0/idx": idx.astype(np.int64), "s0/eps1": EPS_LOG[0], "s0/eps2": EPS_LOG[1]}
    for k, v in tr.get_diagnostics().items():
        out[f"s0/stat/{k}"] = np.array(v, np.float64)
    for gname, opt, order in (("policy", tr.policy_optimizer, PARAM_ORDER_POLICY),
                              ("qf", tr.qf_optimizers[0], PARAM_ORDER_Q)):
        for pname, g, p in zip(order, opt.recorded[-1], opt.param_groups[0]["params"]):
            pack(out, f"s0/grad/{gname}/{pname}", g.numpy(), True)
            st = opt.state[p]
            pack(out, f"s0/adam/{gname}/{pname}/exp_avg", st["exp_avg"].numpy(), False)
            pack(out, f"s0/adam/{gname}/{pname}/exp_avg_sq", st["exp_avg_sq"].numpy(), False)
    out["s0/grad/log_alpha"] = tr.alpha_optimizer.recorded[-1][0].numpy()
    out["s0/post/log_alpha"] = tr.log_alpha.detach().numpy().copy()
    for gname, mod in (("policy", tr.policy), ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
        for pname, tt in mod.state_dict().items():
            pack(out, f"s0/post/{gname}/{pname}", tt.numpy(), False)
    meta = dict(kind="poac", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, K=K, B=B,
                steps=1, n_replay=n_replay, seed=seed, delta=0.95, q_min=q_min, q_max=q_max,
                discount=0.99, lr=lr, tau=tau, idx_seed=idx_seed, eps_seed=eps_seed,
                delta_index=int(tr.delta_index), pi_init_w=1e-3,
                target_entropy=-float(act_dim), counts=False, train_bias=True,
                target_update_period=1, mid_state=dict(t=t, seed=state_seed))
    return meta, out


def gen_mid_all():
    """The BASELINE configs' dims from a mid-training state (one step each)."""
    save("sac_humanoid_mid", *gen_sac_mid("sac_humanoid_mid", 376, 17, [256, 256], 256, 20000))
    save("sac_humanoid_b4096_mid", *gen_sac_mid("sac_humanoid_b4096_mid", 376, 17, [256, 256],
                                                4096, 20000))
    save("poac_ant_b4096_mid", *gen_poac_mid("poac_ant_b4096_mid", 111, 8, [256, 256], 10, 4096,
                                             20000))


# ------------------------------------------------------------- P-OAC runs
def gen_poac(name, obs_dim, act_dim, hidden, K, B, steps, n_replay, full, seed=11,
             delta=0.95, q_min=0.0, q_max=500.0, discount=0.99, lr=3e-4, tau=5e-3,
             idx_seed=1, eps_seed=2, pi_init_w=1e-3, counts=False, train_bias=True, period=1,
             full_s0=False):
    pp, qp = _producers(obs_dim, act_dim, hidden, q_out=K)
    torch.manual_seed(0)
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Box(-1, 1, (act_dim,)),
                            discount=discount, reward_scale=1.0, delta=delta,
                            policy_lr=lr, qf_lr=lr, optimizer_class=Adam14,
                            soft_target_tau=tau, target_update_period=period,
                            use_automatic_entropy_tuning=True, deterministic=False,
                            q_min=q_min, q_max=q_max, share_layers=True, counts=counts,
                            train_bias=train_bias)
    bias = np.linspace(q_min, q_max, K)
    crs = np.random.RandomState(77)   # batch counts (ReplayBufferCount's 'counts' key)
    params = sac_params(obs_dim, act_dim, hidden, seed, q_out=K, q_last_bias=bias,
                        pi_init_w=pi_init_w)
    load_sd(tr.policy, params["policy"])
    load_sd(tr.qfs[0], params["qf1"])
    load_sd(tr.tfs[0], params["target_qf1"])
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    np.random.seed(idx_seed)
    torch.manual_seed(eps_seed)
    out = {}
    meta = dict(kind="poac", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, K=K, B=B,
                steps=steps, n_replay=n_replay, seed=seed, delta=delta, q_min=q_min,
                q_max=q_max, discount=discount, lr=lr, tau=tau, idx_seed=idx_seed,
                eps_seed=eps_seed, delta_index=int(tr.delta_index), pi_init_w=pi_init_w,
                target_entropy=-float(act_dim), counts=counts, train_bias=train_bias,
                target_update_period=period)
    for s in range(steps):
        EPS_LOG.clear()
        batch, idx = _record_batch(rb, B)
        batch = dict(batch)
        if counts:   # about half the rows unvisited (factor 1), the rest 1..3 (:220-224)
            c = crs.randint(0, 4, (B, 1)) * (crs.uniform(0, 1, (B, 1)) < 0.5)
            batch["counts"] = c.astype(np.float64)
            out[f"s{s}/counts"] = batch["counts"][:, 0]
        tr.end_epoch(s)
        tr.train(batch)
        assert len(EPS_LOG) == 2
        out[f"s{s}/idx"] = idx.astype(np.int64)
        out[f"s{s}/eps1"] = EPS_LOG[0]   # drawn by policy(next_obs) (line 193)
        out[f"s{s}/eps2"] = EPS_LOG[1]   # drawn by policy(obs) (line 271)
        for k, v in tr.get_diagnostics().items():
            out[f"s{s}/stat/{k}"] = np.array(v, np.float64)
        for gname, opt, order, mod in (("policy", tr.policy_optimizer, PARAM_ORDER_POLICY,
                                        tr.policy),
                                       ("qf", tr.qf_optimizers[0], PARAM_ORDER_Q, tr.qfs[0])):
            for pname, g in zip(order, opt.recorded[-1]):
                if g is None:   # frozen (train_bias=False)
                    g = torch.zeros_like(mod.state_dict()[pname])
                pack(out, f"s{s}/grad/{gname}/{pname}", g.numpy(), full or (full_s0 and s == 0))
        out[f"s{s}/grad/log_alpha"] = tr.alpha_optimizer.recorded[-1][0].numpy()
        out[f"s{s}/post/log_alpha"] = tr.log_alpha.detach().numpy().copy()
        for gname, mod in (("policy", tr.policy), ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
            for pname, t in mod.state_dict().items():
                pack(out, f"s{s}/post/{gname}/{pname}", t.numpy(), full or (full_s0 and s == 0))
    return meta, out


# ------------------------------------------------------------- g-oac runs
def gen_goac(name, obs_dim, act_dim, hidden, B, steps, n_replay, full, seed=13, delta=0.95,
             r_min=0.0, r_max=5.0, discount=0.99, lr=3e-4, tau=5e-3, idx_seed=1,
             pi_init_w=1e-3, q_init_w=3e-3, counts=False, soft=None, train_bias=True,
             use_target_policy=False):
    """GaussianTrainer (g-oac) as reproduce_g-oac*.sh builds it: share_layers,
    deterministic policy (main.py:219-233), q_min/q_max = r_min/r_max / (1 -
    discount); ``soft``: std_soft_update with that probability.  Parameters
    with no gradient (the deterministic policies' log-std heads) are recorded
    as zero gradients."""
    pp, qp = _producers(obs_dim, act_dim, hidden, q_out=2)
    q_min, q_max = r_min / (1 - discount), r_max / (1 - discount)
    torch.manual_seed(0)
    tr = GaussianTrainer(pp, qp, n_estimators=2, action_space=Box(-1, 1, (act_dim,)),
                         discount=discount, reward_scale=1.0, delta=delta, policy_lr=lr,
                         qf_lr=lr, optimizer_class=Adam14, soft_target_tau=tau,
                         target_update_period=1, q_min=q_min, q_max=q_max, share_layers=True,
                         counts=counts, std_soft_update=soft is not None,
                         std_soft_update_prob=0.0 if soft is None else soft,
                         train_bias=train_bias, use_target_policy=use_target_policy)
    assert tr.deterministic
    params = goac_params(obs_dim, act_dim, hidden, seed, q_min, q_max, pi_init_w=pi_init_w,
                         q_init_w=q_init_w)
    load_sd(tr.policy, params["policy"])
    load_sd(tr.target_policy, params["target_policy"])
    load_sd(tr.q, params["qf1"])
    load_sd(tr.q_target, params["target_qf1"])
    out = {}
    if use_target_policy:   # the DDPG target network: its own weights, recorded
        tpn = goac_params(obs_dim, act_dim, hidden, seed + 100, q_min, q_max,
                          pi_init_w=pi_init_w, q_init_w=q_init_w)["policy"]
        load_sd(tr.target_policy_network, tpn)
        for pname, t in tr.target_policy_network.state_dict().items():
            out[f"tpn/{pname}"] = t.numpy().copy()
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    crs = np.random.RandomState(77)
    np.random.seed(idx_seed)
    meta = dict(kind="goac", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, B=B, steps=steps,
                n_replay=n_replay, seed=seed, delta=delta, q_min=q_min, q_max=q_max,
                discount=discount, lr=lr, tau=tau, idx_seed=idx_seed, pi_init_w=pi_init_w,
                q_init_w=q_init_w, counts=counts, soft=soft, train_bias=train_bias,
                use_target_policy=use_target_policy,
                standard_bound=float(tr.standard_bound), std_init=float(tr.std_init))
    for s in range(steps):
        EPS_LOG.clear()
        batch, idx = _record_batch(rb, B)
        batch = dict(batch)
        if counts:
            c = crs.randint(0, 4, (B, 1)) * (crs.uniform(0, 1, (B, 1)) < 0.5)
            batch["counts"] = c.astype(np.float64)
            out[f"s{s}/counts"] = batch["counts"][:, 0]
        tr.end_epoch(s)
        tr.train(batch)
        assert len(EPS_LOG) == 0      # deterministic policies draw nothing
        out[f"s{s}/idx"] = idx.astype(np.int64)
        for k, v in tr.get_diagnostics().items():
            out[f"s{s}/stat/{k}"] = np.array(v, np.float64)
        for gname, opt, order in (("policy", tr.policy_optimizer, PARAM_ORDER_POLICY),
                                  ("target_policy", tr.target_policy_optimizer,
                                   PARAM_ORDER_POLICY),
                                  ("qf", tr.q_optimizer, PARAM_ORDER_Q)):
            mod = dict(policy=tr.policy, target_policy=tr.target_policy, qf=tr.q)[gname]
            for pname, g in zip(order, opt.recorded[-1]):
                if g is None:
                    g = torch.zeros_like(mod.state_dict()[pname])
                pack(out, f"s{s}/grad/{gname}/{pname}", g.numpy(), full)
        for gname, mod in (("policy", tr.policy), ("target_policy", tr.target_policy),
                           ("qf", tr.q), ("tf", tr.q_target)):
            for pname, t in mod.state_dict().items():
                pack(out, f"s{s}/post/{gname}/{pname}", t.numpy(), full)
    return meta, out


# ------------------------------------------------- p-oac (particle_trainer)
def gen_ptrain(name, obs_dim, act_dim, hidden, K, B, steps, n_replay, full, seed=17, delta=0.95,
               r_min=0.0, r_max=5.0, discount=0.99, lr=3e-4, tau=5e-3, idx_seed=1,
               pi_init_w=1e-3, q_init_w=3e-3, counts=False, soft=None, mean_update=False,
               rescale=False, q_range=None, train_bias=True, use_target_policy=False):
    """ParticleTrainer (trainer/particle_trainer.py) as main.py builds it for
    --alg p-oac without --beta_UB (main.py:198-218): share_layers,
    deterministic policy, q_min/q_max = r_min/r_max / (1 - discount) (or
    ``q_range``).  Parameters with no gradient (the deterministic policies'
    log-std heads) are recorded as zero gradients."""
    pp, qp = _producers(obs_dim, act_dim, hidden, q_out=K)
    q_min, q_max = q_range if q_range else (r_min / (1 - discount), r_max / (1 - discount))
    torch.manual_seed(0)
    tr = ParticleTrainer(pp, qp, n_estimators=K, action_space=Box(-1, 1, (act_dim,)),
                         discount=discount, reward_scale=1.0, delta=delta, policy_lr=lr,
                         qf_lr=lr, optimizer_class=Adam14, soft_target_tau=tau,
                         target_update_period=1, deterministic=True, q_min=q_min, q_max=q_max,
                         share_layers=True, counts=counts, mean_update=mean_update,
                         std_soft_update=soft is not None,
                         std_soft_update_prob=0.0 if soft is None else soft,
                         rescale_targets_around_mean=rescale, train_bias=train_bias,
                         use_target_policy=use_target_policy)
    params = ptrain_params(obs_dim, act_dim, hidden, seed, K, q_min, q_max, pi_init_w=pi_init_w,
                           q_init_w=q_init_w)
    load_sd(tr.policy, params["policy"])
    load_sd(tr.target_policy, params["target_policy"])
    load_sd(tr.qfs[0], params["qf1"])
    load_sd(tr.tfs[0], params["target_qf1"])
    out = {}
    if use_target_policy:   # the DDPG target network: its own weights, recorded
        tpn = ptrain_params(obs_dim, act_dim, hidden, seed + 100, K, q_min, q_max,
                            pi_init_w=pi_init_w, q_init_w=q_init_w)["policy"]
        load_sd(tr.target_policy_network, tpn)
        for pname, t in tr.target_policy_network.state_dict().items():
            out[f"tpn/{pname}"] = t.numpy().copy()
    rb, _ = _fill_buffer(obs_dim, act_dim, n_replay)
    crs = np.random.RandomState(77)
    np.random.seed(idx_seed)
    meta = dict(kind="ptrain", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, K=K, B=B,
                steps=steps, n_replay=n_replay, seed=seed, delta=delta, q_min=q_min,
                q_max=q_max, discount=discount, lr=lr, tau=tau, idx_seed=idx_seed,
                pi_init_w=pi_init_w, q_init_w=q_init_w, counts=counts, soft=soft,
                mean_update=mean_update, rescale=rescale, delta_index=int(tr.delta_index),
                train_bias=train_bias, use_target_policy=use_target_policy)
    for s in range(steps):
        EPS_LOG.clear()
        batch, idx = _record_batch(rb, B)
        batch = dict(batch)
        if counts:
            c = crs.randint(0, 4, (B, 1)) * (crs.uniform(0, 1, (B, 1)) < 0.5)
            batch["counts"] = c.astype(np.float64)
            out[f"s{s}/counts"] = batch["counts"][:, 0]
        tr.end_epoch(s)
        tr.train(batch)
        assert len(EPS_LOG) == 0      # deterministic policies draw nothing
        out[f"s{s}/idx"] = idx.astype(np.int64)
        for k, v in tr.get_diagnostics().items():
            out[f"s{s}/stat/{k}"] = np.array(v, np.float64)
        for gname, opt, mod, order in (
                ("policy", tr.policy_optimizer, tr.policy, PARAM_ORDER_POLICY),
                ("target_policy", tr.target_policy_optimizer, tr.target_policy,
                 PARAM_ORDER_POLICY),
                ("qf", tr.qf_optimizers[0], tr.qfs[0], PARAM_ORDER_Q)):
            for pname, g in zip(order, opt.recorded[-1]):
                if g is None:
                    g = torch.zeros_like(mod.state_dict()[pname])
                pack(out, f"s{s}/grad/{gname}/{pname}", g.numpy(), full)
        for gname, mod in (("policy", tr.policy), ("target_policy", tr.target_policy),
                           ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
            for pname, t in mod.state_dict().items():
                pack(out, f"s{s}/post/{gname}/{pname}", t.numpy(), full)
    return meta, out


def gen_ptrain_all():
    save("ptrain_small", *gen_ptrain("ptrain_small", 111, 8, [32, 32], 10, 32, 3, 500, True,
                                     pi_init_w=0.3, q_init_w=0.3))
    save("ptrain_counts", *gen_ptrain("ptrain_counts", 111, 8, [32, 32], 10, 32, 3, 500, True,
                                      pi_init_w=0.3, q_init_w=0.3, counts=True))
    save("ptrain_soft_rescale", *gen_ptrain("ptrain_soft_rescale", 11, 3, [16, 16], 5, 16, 3,
                                            200, True, pi_init_w=0.5, q_init_w=0.5, soft=0.3,
                                            rescale=True, q_range=(0.0, 1.0), lr=1e-3,
                                            tau=0.05, delta=0.75))
    save("ptrain_mean_update", *gen_ptrain("ptrain_mean_update", 11, 3, [16, 16], 10, 16, 3, 200,
                                           True, pi_init_w=0.5, q_init_w=0.5, mean_update=True,
                                           lr=1e-3))
    save("ptrain_humanoid", *gen_ptrain("ptrain_humanoid", 376, 17, [256, 256], 10, 256, 2,
                                        20000, False, counts=True))


# ------------------------------------------------------- OAC exploration
def gen_oac_expl(name, obs_dim, act_dim, hidden, n_obs, beta_UB, delta, seed=5,
                 pi_init_w=0.1, q_init_w=0.1, eps_seed=3, K=None, ub_delta=None):
    """K: one shared-layer critic with K heads (share_layers=True, the except
    branch of optimistic_exploration.py:47-56) instead of twin critics.
    ub_delta: additionally pass trainer= a particle_trainer_oac.ParticleTrainer
    built with delta=ub_delta (--trainer_UB: Q_UB = trainer.predict, the
    sorted head delta_index, particle_trainer_oac.py:147-167)."""
    pp, qp = _producers(obs_dim, act_dim, hidden, q_out=K or 1)
    policy = pp()
    params = sac_params(obs_dim, act_dim, hidden, seed, pi_init_w=pi_init_w, q_init_w=q_init_w,
                        q_out=K or 1,
                        q_last_bias=None if K is None else np.linspace(0.0, 50.0, K))
    load_sd(policy, params["policy"])
    qf1 = qp()
    load_sd(qf1, params["qf1"])
    trainer, delta_index = None, None
    if ub_delta is not None:
        torch.manual_seed(0)
        trainer = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Box(-1, 1, (act_dim,)),
                                     delta=ub_delta, optimizer_class=Adam14, q_min=0.0,
                                     q_max=50.0, share_layers=True, deterministic=False)
        load_sd(trainer.policy, params["policy"])
        load_sd(trainer.qfs[0], params["qf1"])
        policy, qf1 = trainer.policy, trainer.qfs[0]
        delta_index = int(trainer.delta_index)
    if K is None:
        qf2 = qp()
        load_sd(qf2, params["qf2"])
        qfs = [qf1, qf2]
    else:
        qfs = [qf1]
    rs = np.random.RandomState(seed + 100)
    obs = rs.standard_normal((n_obs, obs_dim))  # float64, like env observations
    captured = []
    orig_tn = oe.TanhNormal

    class CapTN(orig_tn):
        def __init__(self, mean, std, *a, **k):
            captured.append((mean.detach().numpy().copy(), std.detach().numpy().copy()))
            super().__init__(mean, std, *a, **k)

    oe.TanhNormal = CapTN
    torch.manual_seed(eps_seed)
    out = {"obs": obs}
    acts, mu_e, stds, eps_d, eps_s = [], [], [], [], []
    hp = dict(beta_UB=beta_UB, delta=delta, share_layers=K is not None)
    try:
        for i in range(n_obs):
            EPS_LOG.clear()
            captured.clear()
            a, info = oe.get_optimistic_exploration_action(obs[i], policy=policy, qfs=qfs,
                                                           trainer=trainer, hyper_params=hp)
            assert len(EPS_LOG) == 2 and len(captured) == 1
            eps_d.append(EPS_LOG[0])
            eps_s.append(EPS_LOG[1])
            mu_e.append(captured[0][0])
            stds.append(captured[0][1])
            acts.append(np.asarray(a, np.float32))
    finally:
        oe.TanhNormal = orig_tn
    out.update(action=np.stack(acts), mu_E=np.stack(mu_e), std=np.stack(stds),
               eps_discard=np.stack(eps_d), eps=np.stack(eps_s))
    meta = dict(kind="oac_expl", obs_dim=obs_dim, act_dim=act_dim, hidden=hidden, n_obs=n_obs,
                beta_UB=beta_UB, delta=delta, seed=seed, pi_init_w=pi_init_w, q_init_w=q_init_w,
                K=K, ub_delta=ub_delta, delta_index=delta_index)
    return meta, out


# -------------------------------------------------------- numpy randint
def gen_randint():
    """Legacy MT19937 ``np.random.randint(0, size, B)`` streams, exactly as
    ``ReplayBuffer.random_batch`` calls it (replay_buffer.py:107)."""
    cases = [(1, 1000, 256), (1, 10000, 256), (2, 1000000, 4096), (3, 1, 64),
             (4, 2 ** 20, 1000), (5, 2 ** 20 + 1, 1000), (6, 3, 2000), (7, 2, 100),
             (8, 4294967295, 50), (9, 123457, 4096), (0, 2 ** 31, 300)]
    out = {}
    for n, (seed, size, B) in enumerate(cases):
        np.random.seed(seed)
        a = np.random.randint(0, size, B)
        b = np.random.randint(0, size, B)   # continuity across calls
        c = np.random.randint(0, 1, 7)      # rng == 0: no draw consumed
        d = np.random.randint(0, size, B)
        out[f"c{n}/seed"] = np.array(seed)
        out[f"c{n}/size"] = np.array(size, np.int64)
        out[f"c{n}/B"] = np.array(B)
        out[f"c{n}/idx"] = np.concatenate([a, b, c, d]).astype(np.int64)
    return dict(kind="randint", n_cases=len(cases)), out


# ------------------------------------------------- ReplayBufferCount
def _path(rs, T, obs_dim, act_dim):
    """One rollout path in the reference's layout (path_collector.py rollout)."""
    return dict(observations=rs.standard_normal((T, obs_dim)) * 3.0,
                actions=rs.uniform(-1, 1, (T, act_dim)),
                rewards=rs.standard_normal((T, 1)) * 10.0,
                next_observations=rs.standard_normal((T, obs_dim)) * 3.0,
                terminals=(rs.uniform(0, 1, (T, 1)) < 0.1),
                agent_infos=[{}] * T, env_infos=[{}] * T)


def gen_replay_count(priority):
    """ReplayBufferCount (replay_buffer.py:151-197) run by the reference:
    add_paths that wrap the ring, random_batch with the counts bookkeeping
    (and np.random.choice priority sampling), recording per call the indices
    (recomputed from the saved global RNG state with the reference's own
    numpy algorithm and checked against the returned rows), the batch's
    counts and the counts array after the update."""
    obs_dim, act_dim, N, B = 5, 2, 600, 64
    rb = ReplayBufferCount(N, Box(-1, 1, (obs_dim,)), Box(-1, 1, (act_dim,)),
                           priority_sample=priority)
    rs = np.random.RandomState(21)
    np.random.seed(33)
    out, ops = {}, []
    for k in range(12):
        T = int(rs.randint(20, 160))
        path = _path(rs, T, obs_dim, act_dim)
        rb.add_paths([path])
        for key in ("observations", "actions", "rewards", "next_observations", "terminals"):
            out[f"op{k}/path/{key}"] = np.asarray(path[key])
        st = np.random.get_state()
        batch = rb.random_batch(B)
        r2 = np.random.RandomState()
        r2.set_state(st)
        if priority:
            u = r2.random_sample(B)
            out[f"op{k}/u"] = u
        out[f"op{k}/counts_batch"] = batch["counts"][:, 0].astype(np.int64)
        out[f"op{k}/counts_after"] = rb._counts[:, 0].astype(np.int64).copy()
        out[f"op{k}/obs"] = batch["observations"]
        ops.append(T)
    out["final/observations"] = rb._observations
    out["final/actions"] = rb._actions
    out["final/rewards"] = rb._rewards
    out["final/terminals"] = rb._terminals
    out["final/next_obs"] = rb._next_obs
    out["final/top_size"] = np.array([rb._top, rb._size])
    meta = dict(kind="replay_count", priority=priority, obs_dim=obs_dim, act_dim=act_dim, N=N,
                B=B, path_lengths=ops, np_seed=33)
    return meta, out


# ------------------------------------------------------------ checkpoint
def _plain(x):
    """A snapshot in types torch.load(weights_only=True) accepts."""
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_plain(v) for v in x)
    if isinstance(x, torch.Tensor):
        return x.detach().clone()
    if isinstance(x, np.generic):
        return x.item()
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x.copy())
    return x


def gen_sac_snapshot(path, obs_dim=11, act_dim=3, hidden=(32, 32), B=16, seed=7):
    """The reference SACTrainer's checkpoint (trainer/trainer.py:299-317,
    restored by :319-369) after two steps, and the third step it then takes:
    its batch indices, eps draws and the post-step parameters."""
    pp, qp = _producers(obs_dim, act_dim, list(hidden))
    torch.manual_seed(0)
    tr = SACTrainer(pp, qp, action_space=Box(-1, 1, (act_dim,)), discount=0.99, reward_scale=1.0,
                    policy_lr=3e-4, qf_lr=3e-4, optimizer_class=Adam14, soft_target_tau=5e-3,
                    target_update_period=1, use_automatic_entropy_tuning=True)
    params = sac_params(obs_dim, act_dim, list(hidden), seed, pi_init_w=0.2, q_init_w=0.1)
    load_sd(tr.policy, params["policy"])
    for k in ("qf1", "qf2", "target_qf1", "target_qf2"):
        load_sd(getattr(tr, k), params[k])
    rb, _ = _fill_buffer(obs_dim, act_dim, 300)
    np.random.seed(3)
    torch.manual_seed(4)
    for s in range(2):
        batch, _ = _record_batch(rb, B)
        tr.end_epoch(s)
        tr.train(dict(batch))
    snap = _plain(tr.get_snapshot())
    EPS_LOG.clear()
    batch, idx = _record_batch(rb, B)
    tr.end_epoch(2)
    tr.train(dict(batch))
    post = {g: {k: v.detach().clone() for k, v in getattr(tr, g).state_dict().items()}
            for g in ("policy", "qf1", "qf2", "target_qf1", "target_qf2")}
    fixture = dict(meta=dict(obs_dim=obs_dim, act_dim=act_dim, hidden=list(hidden), B=B, seed=seed,
                             pi_init_w=0.2, q_init_w=0.1, n_replay=300, lr=3e-4, tau=5e-3),
                   snapshot=snap, step3=dict(idx=torch.from_numpy(idx.astype(np.int64)),
                                             eps1=torch.from_numpy(EPS_LOG[0]),
                                             eps2=torch.from_numpy(EPS_LOG[1]), post=post,
                                             log_alpha=tr.log_alpha.detach().clone()))
    torch.save(fixture, path)
    print(f"{os.path.basename(path)}: {os.path.getsize(path) / 1e3:.0f} KB")


def gen_det_snapshot(path, kind, obs_dim=11, act_dim=3, hidden=(32, 32), B=16, seed=9):
    """A checkpoint of the reference's GaussianTrainer (kind 'goac') or
    particle_trainer.ParticleTrainer (kind 'ptrain', K=5) after two counts=True
    steps -- built as main.py builds them (use_automatic_entropy_tuning from
    --entropy_tuning, default on, so the snapshot carries log_alpha and the
    unused alpha optimizer; gaussian_trainer.py:452-482,
    particle_trainer.py:449-478) -- and the third step it then takes."""
    K = 2 if kind == "goac" else 5
    pp, qp = _producers(obs_dim, act_dim, list(hidden), q_out=K)
    torch.manual_seed(0)
    common = dict(action_space=Box(-1, 1, (act_dim,)), discount=0.99, reward_scale=1.0,
                  delta=0.95, policy_lr=3e-4, qf_lr=3e-4, optimizer_class=Adam14,
                  soft_target_tau=5e-3, target_update_period=1,
                  use_automatic_entropy_tuning=True, q_min=0.0, q_max=100.0,
                  share_layers=True, counts=True)
    if kind == "goac":
        tr = GaussianTrainer(pp, qp, n_estimators=2, **common)
        params = goac_params(obs_dim, act_dim, list(hidden), seed, 0.0, 100.0, pi_init_w=0.2,
                             q_init_w=0.1)
        qf, tf = tr.q, tr.q_target
    else:
        tr = ParticleTrainer(pp, qp, n_estimators=K, deterministic=True, **common)
        params = ptrain_params(obs_dim, act_dim, list(hidden), seed, K, 0.0, 100.0,
                               pi_init_w=0.2, q_init_w=0.1)
        qf, tf = tr.qfs[0], tr.tfs[0]
    load_sd(tr.policy, params["policy"])
    load_sd(tr.target_policy, params["target_policy"])
    load_sd(qf, params["qf1"])
    load_sd(tf, params["target_qf1"])
    rb, _ = _fill_buffer(obs_dim, act_dim, 300)
    crs = np.random.RandomState(5)
    np.random.seed(3)

    def batch_with_counts():
        batch, idx = _record_batch(rb, B)
        batch = dict(batch)
        batch["counts"] = (crs.randint(0, 3, (B, 1)) * (crs.uniform(0, 1, (B, 1)) < 0.5)
                           ).astype(np.float64)
        return batch, idx
    for s in range(2):
        batch, _ = batch_with_counts()
        tr.end_epoch(s)
        tr.train(batch)
    snap = _plain(tr.get_snapshot())
    batch, idx = batch_with_counts()
    tr.end_epoch(2)
    tr.train(dict(batch))
    mods = dict(policy=tr.policy, target_policy=tr.target_policy, qf=qf, tf=tf)
    post = {g: {k: v.detach().clone() for k, v in m.state_dict().items()} for g, m in mods.items()}
    fixture = dict(meta=dict(kind=kind, obs_dim=obs_dim, act_dim=act_dim, hidden=list(hidden), B=B,
                             K=K, seed=seed, pi_init_w=0.2, q_init_w=0.1, n_replay=300, lr=3e-4,
                             tau=5e-3, q_min=0.0, q_max=100.0, delta=0.95, discount=0.99),
                   snapshot=snap,
                   step3=dict(idx=torch.from_numpy(idx.astype(np.int64)),
                              counts=torch.from_numpy(batch["counts"]), post=post))
    torch.save(fixture, path)
    print(f"{os.path.basename(path)}: {os.path.getsize(path) / 1e3:.0f} KB")


def gen_period():
    """target_update_period = 2 (trainer/trainer.py:215, particle_trainer_oac.py:
    320): Polyak only on even steps; tau 0.1 so the skipped updates show."""
    save("sac_period2", *gen_sac("sac_period2", 11, 3, [32, 32], 16, 4, 300, True, tau=0.1,
                                 lr=1e-3, pi_init_w=0.2, q_init_w=0.1, period=2))
    save("poac_period2", *gen_poac("poac_period2", 11, 3, [32, 32], 5, 16, 4, 300, True,
                                   tau=0.1, lr=1e-3, q_max=50.0, period=2))


def save(name, meta, out):
    import json
    out = dict(out)
    out["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {os.path.getsize(path) / 1e3:.0f} KB, {len(out)} arrays")


def gen_tpn():
    """use_target_policy (the DDPG target network, particle_trainer.py:150-154,
    196-199, 386-388; gaussian_trainer.py the same): next actions from a
    separate policy network that the reference's soft update never moves."""
    save("ptrain_tpn", *gen_ptrain("ptrain_tpn", 11, 3, [16, 16], 5, 16, 3, 200, True,
                                   pi_init_w=0.5, q_init_w=0.5, lr=1e-3,
                                   use_target_policy=True))
    save("goac_tpn", *gen_goac("goac_tpn", 11, 3, [16, 16], 16, 3, 200, True, pi_init_w=0.5,
                               q_init_w=0.5, lr=1e-3, use_target_policy=True))


def main():
    torch.set_num_threads(8)
    if len(sys.argv) > 1 and sys.argv[1] == "period":
        gen_period()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sac_snapshot":
        gen_sac_snapshot(os.path.join(HERE, "sac_snapshot.pt"))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "poac_counts":
        save("poac_counts", *gen_poac("poac_counts", 111, 8, [32, 32], 10, 32, 2, 500, True,
                                      pi_init_w=0.3, counts=True))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "humanoid":
        gen_humanoid()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "mid":
        gen_mid_all()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "poac_b4096":
        gen_poac_b4096()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "nobias":
        gen_nobias()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "oac_expl_shared":
        gen_expl_shared()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "oac_expl_trainer_ub":
        gen_expl_trainer_ub()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "det_snapshot":
        gen_det_snapshot(os.path.join(HERE, "goac_snapshot.pt"), "goac")
        gen_det_snapshot(os.path.join(HERE, "ptrain_snapshot.pt"), "ptrain")
        return
    if len(sys.argv) > 1 and sys.argv[1] == "ptrain":
        gen_ptrain_all()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "target_policy_network":
        gen_tpn()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "goac":
        gen_goac_all()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "replay_count":
        save("replay_count", *gen_replay_count(False))
        save("replay_count_priority", *gen_replay_count(True))
        return
    save("randint", *gen_randint())
    save("sac_small", *gen_sac("sac_small", 376, 17, [32, 32], 32, 3, 1000, True))
    save("sac_stress", *gen_sac("sac_stress", 11, 3, [32, 32], 16, 3, 300, True,
                                pi_init_w=0.7, q_init_w=0.3, log_alpha0=-0.5,
                                discount=0.95, reward_scale=2.0, tau=0.01, lr=1e-3))
    save("sac_noalpha", *gen_sac("sac_noalpha", 5, 2, [16, 16], 8, 2, 100, True,
                                 auto_alpha=False, pi_init_w=0.2))
    save("sac_riverswim", *gen_sac("sac_riverswim", 1, 1, [256, 256], 256, 2, 10000, False))
    gen_humanoid()
    save("poac_small", *gen_poac("poac_small", 111, 8, [32, 32], 10, 32, 2, 500, True,
                                 pi_init_w=0.3))
    save("poac_ant", *gen_poac("poac_ant", 111, 8, [256, 256], 10, 512, 2, 20000, False))
    save("oac_expl_humanoid", *gen_oac_expl("oac_expl_humanoid", 376, 17, [256, 256], 16,
                                            4.66, 23.53))
    save("oac_expl_small", *gen_oac_expl("oac_expl_small", 11, 3, [32, 32], 16, 0.0, 5.0))
    save("replay_count", *gen_replay_count(False))
    save("replay_count_priority", *gen_replay_count(True))
    save("poac_counts", *gen_poac("poac_counts", 111, 8, [32, 32], 10, 32, 2, 500, True,
                                  pi_init_w=0.3, counts=True))
    gen_sac_snapshot(os.path.join(HERE, "sac_snapshot.pt"))
    gen_goac_all()
    gen_ptrain_all()
    gen_det_snapshot(os.path.join(HERE, "goac_snapshot.pt"), "goac")
    gen_det_snapshot(os.path.join(HERE, "ptrain_snapshot.pt"), "ptrain")
    gen_expl_shared()
    gen_nobias()


def gen_humanoid():
    """The headline configs (BASELINE configs[1] / [2] dims): step 0 whole."""
    save("sac_humanoid", *gen_sac("sac_humanoid", 376, 17, [256, 256], 256, 3, 20000, False,
                                  full_s0=True))
    save("sac_humanoid_b4096", *gen_sac("sac_humanoid_b4096", 376, 17, [256, 256], 4096, 3,
                                        20000, False, full_s0=True))


def gen_poac_b4096():
    """BASELINE configs[4] at its own batch: K=10 shared-head critic, Ant-v2
    dims, 2x256, B=4096, two steps, step 0 whole."""
    save("poac_ant_b4096", *gen_poac("poac_ant_b4096", 111, 8, [256, 256], 10, 4096, 2, 20000,
                                     False, full_s0=True))


def gen_nobias():
    """train_bias=False (--no_train_bias): the critics' last-layer bias is frozen."""
    save("poac_nobias", *gen_poac("poac_nobias", 11, 3, [16, 16], 5, 16, 3, 200, True,
                                  pi_init_w=0.3, train_bias=False))
    save("goac_nobias", *gen_goac("goac_nobias", 11, 3, [16, 16], 16, 3, 200, True,
                                  pi_init_w=0.5, q_init_w=0.5, train_bias=False, counts=True))
    save("ptrain_nobias", *gen_ptrain("ptrain_nobias", 11, 3, [16, 16], 5, 16, 3, 200, True,
                                      pi_init_w=0.5, q_init_w=0.5, train_bias=False, counts=True))


def gen_expl_shared():
    save("oac_expl_shared_ant", *gen_oac_expl("oac_expl_shared_ant", 111, 8, [256, 256], 16,
                                              4.66, 23.53, K=10, q_init_w=0.3))
    save("oac_expl_shared_small", *gen_oac_expl("oac_expl_shared_small", 11, 3, [32, 32], 16,
                                                2.0, 5.0, K=4, q_init_w=0.5))


def gen_expl_trainer_ub():
    save("oac_expl_ub_ant", *gen_oac_expl("oac_expl_ub_ant", 111, 8, [256, 256], 16,
                                          4.66, 23.53, K=10, q_init_w=0.3, ub_delta=0.6))
    save("oac_expl_ub_small", *gen_oac_expl("oac_expl_ub_small", 11, 3, [32, 32], 16,
                                            2.0, 5.0, K=4, q_init_w=0.5, ub_delta=0.75))


def gen_goac_all():
    save("goac_small", *gen_goac("goac_small", 111, 8, [32, 32], 32, 3, 500, True,
                                 pi_init_w=0.3, q_init_w=0.3))
    save("goac_counts", *gen_goac("goac_counts", 111, 8, [32, 32], 32, 3, 500, True,
                                  pi_init_w=0.3, q_init_w=0.3, counts=True))
    save("goac_soft", *gen_goac("goac_soft", 11, 3, [16, 16], 16, 3, 200, True,
                                pi_init_w=0.5, q_init_w=0.5, soft=0.3, r_min=-1.0, r_max=1.0,
                                discount=0.9, tau=0.05, lr=1e-3))
    save("goac_humanoid", *gen_goac("goac_humanoid", 376, 17, [256, 256], 256, 2, 20000, False,
                                    counts=True))


if __name__ == "__main__":
    main()
