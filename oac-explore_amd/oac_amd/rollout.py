"""Rollouts that feed the exploration call.

``rollout`` keeps the contract of path_collector.rollout
(/root/reference/path_collector.py:176-257): one environment, one
``get_optimistic_exploration_action`` (or ``agent.get_action``) per step, and
the same path dict (observations, actions, rewards, next_observations,
terminals as 2-D arrays; agent_infos / env_infos as per-step lists).

``vec_rollout`` steps N environments in lockstep and computes the actions of
all still-running environments with ONE call per step
(``get_optimistic_exploration_actions``, or ``agent.get_actions``), returning
N path dicts with exactly ``rollout``'s layout.  With the exploration noise
fixed (``optimistic_exploration_kwargs['eps']``) every path is bitwise the
path ``rollout`` collects from the same environment; with device Philox noise
the draws of a step come from one counter value (rows r*Da .. r*Da+Da-1), so
the paths are the same in distribution, not draw for draw.
"""
import numpy as np

from .optimistic_exploration import (get_optimistic_exploration_action,
                                     get_optimistic_exploration_actions)


def _path(observations, actions, rewards, terminals, agent_infos, env_infos, next_o):
    """path_collector.py:238-257: stack the per-step lists."""
    actions = np.array(actions)
    if len(actions.shape) == 1:
        actions = np.expand_dims(actions, 1)
    observations = np.array(observations)
    if len(observations.shape) == 1:
        observations = np.expand_dims(observations, 1)
        next_o = np.array([next_o])
    next_observations = np.vstack((observations[1:, :], np.expand_dims(next_o, 0)))
    return dict(
        observations=observations,
        actions=actions,
        rewards=np.array(rewards).reshape(-1, 1),
        next_observations=next_observations,
        terminals=np.array(terminals).reshape(-1, 1),
        agent_infos=agent_infos,
        env_infos=env_infos,
    )


def rollout(env, agent, max_path_length=np.inf, render=False, render_kwargs=None,
            optimistic_exploration=False, optimistic_exploration_kwargs={},
            deterministic_pol=False):
    """path_collector.rollout (path_collector.py:176-257) on the HIP exploration
    call: same arguments, same loop (reset, act, step, stop at a terminal or
    max_path_length), same returned dict."""
    if render_kwargs is None:
        render_kwargs = {}
    observations, actions, rewards, terminals, agent_infos, env_infos = [], [], [], [], [], []
    o = env.reset()
    agent.reset()
    next_o = None
    path_length = 0
    if render:
        env.render(**render_kwargs)
    while path_length < max_path_length:
        if not optimistic_exploration:
            a, agent_info = agent.get_action(o, deterministic=deterministic_pol)
        else:
            a, agent_info = get_optimistic_exploration_action(o, **optimistic_exploration_kwargs)
        next_o, r, d, env_info = env.step(a)
        observations.append(o)
        rewards.append(r)
        terminals.append(d)
        actions.append(a)
        agent_infos.append(agent_info)
        env_infos.append(env_info)
        path_length += 1
        if d:
            break
        o = next_o
        if render:
            env.render(**render_kwargs)
    return _path(observations, actions, rewards, terminals, agent_infos, env_infos, next_o)


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
    """``rollout`` over N environments with one batched action call per step.
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
    return [_path(b["o"], b["a"], b["r"], b["d"], b["ai"], b["ei"], last[i])
            for i, b in enumerate(buf)]
