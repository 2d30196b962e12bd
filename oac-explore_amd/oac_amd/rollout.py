"""Vectorised rollouts that feed the exploration call.

The single-environment loop stays the reference's own
``path_collector.rollout`` (/root/reference/path_collector.py:176-257): with
``get_optimistic_exploration_action`` imported from ``oac_amd`` instead of
``optimistic_exploration`` it runs on the HIP exploration
kernel unchanged.

``vec_rollout`` steps N environments in lockstep and computes the actions of
all still-running environments with ONE call per step
(``get_optimistic_exploration_actions``, or ``agent.get_actions``), returning
N path dicts in ``path_collector.rollout``'s layout (observations, actions,
rewards, next_observations, terminals as 2-D arrays; agent_infos / env_infos
as per-step lists).  With the exploration noise fixed
(``optimistic_exploration_kwargs['eps']``) every path is bitwise the path the
single-environment loop collects from the same environment; with device
Philox noise the draws of a step come from one counter value (rows r*Da ..
r*Da+Da-1), so the paths are the same in distribution, not draw for draw.
"""
import numpy as np

from .optimistic_exploration import get_optimistic_exploration_actions


def _as_rows(x):
    """Per-step values stacked as rows: [T] -> [T, 1], [T, d] unchanged."""
    x = np.asarray(x)
    return x.reshape(len(x), -1) if x.ndim <= 1 else x


def _pack(rec, last_obs):
    """One environment's record as the path dict path_collector.rollout
    returns: next_observations are the observations shifted by one with the
    final next observation appended."""
    obs = _as_rows(rec["o"])
    tail = np.asarray(last_obs).reshape(1, -1)
    return {"observations": obs,
            "actions": _as_rows(rec["a"]),
            "rewards": np.asarray(rec["r"]).reshape(-1, 1),
            "next_observations": np.concatenate([obs[1:], tail], axis=0),
            "terminals": np.asarray(rec["d"]).reshape(-1, 1),
            "agent_infos": rec["ai"],
            "env_infos": rec["ei"]}


def _batch_actions(agent, obs, optimistic_exploration, kwargs, deterministic_pol):
    """Actions [n, Da] and per-row agent infos for the running environments."""
    n = obs.shape[0]
    if optimistic_exploration:
        kw = dict(kwargs)
        eps = kw.pop("eps", None)
        if eps is not None:
            eps = np.asarray(eps, np.float32)
            if eps.ndim == 1:
                eps = np.tile(eps, (n, 1))   # writable (torch.from_numpy of a view warns)
        kw.pop("deterministic", None)
        A, _ = get_optimistic_exploration_actions(obs, eps=eps, **kw)
        return A, [{} for _ in range(n)]
    if hasattr(agent, "stochastic_policy"):          # MakeDeterministic (policies.py:486-513)
        A = agent.get_actions(obs)
    else:
        A = agent.get_actions(obs, deterministic=deterministic_pol)
    return np.asarray(A), [{} for _ in range(n)]


def vec_rollout(envs, agent, max_path_length=np.inf, optimistic_exploration=False,
                optimistic_exploration_kwargs={}, deterministic_pol=False):
    """path_collector.rollout over N environments with one batched action call per step.
    Returns one path dict per environment (in the order of ``envs``); an
    environment leaves the batch at its first terminal or at max_path_length."""
    n_env = len(envs)
    obs = [env.reset() for env in envs]
    agent.reset()
    buf = [dict(o=[], a=[], r=[], d=[], ai=[], ei=[]) for _ in range(n_env)]
    last = [None] * n_env
    running = list(range(n_env))
    t = 0
    while running and t < max_path_length:
        O = np.stack([np.asarray(obs[i]) for i in running])
        A, infos = _batch_actions(agent, O, optimistic_exploration, optimistic_exploration_kwargs,
                                  deterministic_pol)
        still = []
        for row, i in enumerate(running):
            a = A[row]
            next_o, r, d, env_info = envs[i].step(a)
            b = buf[i]
            b["o"].append(obs[i]); b["a"].append(a); b["r"].append(r); b["d"].append(d)
            b["ai"].append(infos[row]); b["ei"].append(env_info)
            last[i] = next_o
            if not d:
                obs[i] = next_o
                still.append(i)
        running = still
        t += 1
    return [_pack(b, last[i]) for i, b in enumerate(buf)]
