"""vec_rollout (oac_amd/rollout.py) against the contract of
path_collector.rollout (/root/reference/path_collector.py:176-257): the path
dict layout (2-D observations / actions / rewards / next_observations /
terminals, per-step info lists), terminal / max_path_length handling, and --
with a deterministic agent on the CPU, or fixed exploration noise on the GPU
-- every environment's path equal to stepping that environment alone with one
single-observation action call per step (`walk` below)."""
import numpy as np
import pytest


class ToyEnv:
    """Observations depend on the actions (so a wrong action shows up in every
    later row); done after `length` steps."""

    def __init__(self, obs_dim, length, seed):
        self.obs_dim, self.length, self.seed = obs_dim, length, seed

    def reset(self):
        self.t = 0
        self.o = np.random.RandomState(self.seed).standard_normal(self.obs_dim)
        return self.o.copy()

    def step(self, a):
        self.t += 1
        a = np.asarray(a, np.float64)
        self.o = np.tanh(self.o + np.resize(a, self.obs_dim) * 0.5)
        return self.o.copy(), float(a.sum()), self.t >= self.length, {"t": self.t}


class LinearAgent:
    def __init__(self, obs_dim, act_dim):
        self.W = np.random.RandomState(7).standard_normal((act_dim, obs_dim)) * 0.3

    def reset(self):
        pass

    def get_action(self, o, deterministic=False):
        return np.tanh(self.W @ o).astype(np.float32), {}

    def get_actions(self, O, deterministic=False):
        return np.tanh(O @ self.W.T).astype(np.float32)


def walk(env, act, max_path_length):
    """One environment stepped alone: act(o) -> action per step; the
    transitions it saw, as arrays."""
    O, A, R, D, E = [], [], [], [], []
    o = env.reset()
    while len(O) < max_path_length:
        a = act(o)
        o2, r, d, info = env.step(a)
        O.append(o); A.append(a); R.append(r); D.append(d); E.append(info)
        o = o2
        if d:
            break
    return dict(observations=np.array(O), actions=np.array(A),
                rewards=np.array(R).reshape(-1, 1),
                next_observations=np.vstack([np.array(O[1:]).reshape(-1, len(o)), o[None]]),
                terminals=np.array(D).reshape(-1, 1), env_infos=E, agent_infos=[{}] * len(O))


def _same(p, q):
    for k in ("observations", "actions", "rewards", "next_observations", "terminals"):
        assert p[k].shape == q[k].shape, k
        np.testing.assert_array_equal(p[k], q[k], err_msg=k)
    assert p["env_infos"] == q["env_infos"]
    assert len(p["agent_infos"]) == len(q["agent_infos"])


def test_vec_rollout_equals_single_env_walks_cpu_agent():
    from oac_amd.rollout import vec_rollout
    Do, Da = 5, 3
    lengths = [1, 4, 9, 12]
    agent = LinearAgent(Do, Da)
    paths = vec_rollout([ToyEnv(Do, L, s) for s, L in enumerate(lengths)], agent,
                        max_path_length=10)
    for s, L in enumerate(lengths):
        ref = walk(ToyEnv(Do, L, s), lambda o: agent.get_action(o)[0], 10)
        _same(paths[s], ref)
        p = paths[s]
        assert all(p[k].ndim == 2 for k in ("observations", "actions", "rewards",
                                            "next_observations", "terminals"))
        assert len(p["observations"]) == min(L, 10)
        assert p["terminals"][-1, 0] == (L <= 10)
        np.testing.assert_array_equal(p["next_observations"][:-1], p["observations"][1:])


def test_vec_rollout_scalar_observations():
    """1-D environments (riverswim: obs 1, act 1): observations, actions and
    next_observations still come back as [T, 1]."""
    from oac_amd.rollout import vec_rollout

    class Scalar:
        def __init__(self, L):
            self.L = L

        def reset(self):
            self.t, self.o = 0, 0.5
            return self.o

        def step(self, a):
            self.t += 1
            self.o = float(np.tanh(self.o + float(np.asarray(a).reshape(-1)[0])))
            return self.o, self.o, self.t >= self.L, {}

    class Agent:
        def reset(self):
            pass

        def get_actions(self, O, deterministic=False):
            return (0.3 * np.asarray(O, np.float32)).reshape(-1, 1)

    paths = vec_rollout([Scalar(3), Scalar(5)], Agent(), max_path_length=4)
    for p, T in zip(paths, (3, 4)):
        for k in ("observations", "actions", "rewards", "next_observations", "terminals"):
            assert p[k].shape == (T, 1), (k, p[k].shape)
        np.testing.assert_array_equal(p["next_observations"][:-1], p["observations"][1:])


@pytest.mark.gpu
def test_vec_rollout_oac_equals_single_env_walks():
    """OAC exploration with fixed noise: the batched call per step reproduces
    every single-environment path bitwise (the action rows of a batched call
    are bitwise the single calls)."""
    import torch
    from oac_amd import get_optimistic_exploration_action
    from oac_amd.rollout import vec_rollout
    from gpu_helpers import Space
    import oac_amd
    Do, Da, H = 11, 3, [32, 32]
    dev = torch.device("cuda", 0)
    tr = oac_amd.SACTrainer(oac_amd.get_policy_producer(Do, Da, H, device=dev),
                            oac_amd.get_q_producer(Do, Da, H, device=dev),
                            action_space=Space(Da), device=dev)
    kw = dict(policy=tr.policy, qfs=tr.qfs, hyper_params=dict(beta_UB=4.66, delta=23.53),
              eps=np.full(Da, 0.25, np.float32))
    lengths = [3, 7, 7, 20]
    paths = vec_rollout([ToyEnv(Do, L, 10 + s) for s, L in enumerate(lengths)], tr.policy,
                        max_path_length=16, optimistic_exploration=True,
                        optimistic_exploration_kwargs=kw)
    for s, L in enumerate(lengths):
        ref = walk(ToyEnv(Do, L, 10 + s),
                   lambda o: get_optimistic_exploration_action(o, **kw)[0], 16)
        _same(paths[s], ref)
    # plain policy actions (no exploration): batched get_actions vs get_action
    paths = vec_rollout([ToyEnv(Do, L, s) for s, L in enumerate(lengths)], tr.policy,
                        max_path_length=5, deterministic_pol=True)
    for s, L in enumerate(lengths):
        ref = walk(ToyEnv(Do, L, s), lambda o: tr.policy.get_action(o, deterministic=True)[0], 5)
        for k in ("observations", "actions", "rewards"):
            np.testing.assert_allclose(paths[s][k], ref[k], rtol=1e-6, atol=1e-6)
