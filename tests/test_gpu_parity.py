"""GPU parity: the HIP path (through the C ABI) against the golden fixtures the
reference produced and against the CPU oracle on the same inputs."""
import numpy as np
import pytest
import torch

import parity
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q, sac_params, synthetic_transitions
from gpu_helpers import batch_from, module_tensors, sac_trainer_for
from oracle import sac_oracle as so

pytestmark = pytest.mark.gpu

SAC_FIXTURES = ["sac_small", "sac_stress", "sac_noalpha", "sac_riverswim", "sac_humanoid",
                "sac_humanoid_b4096", "sac_period2"]


def _oracle_noise(meta, g):
    """per-key fp32 noise of the trajectory (test_oracle_golden.noise_of)."""
    import test_oracle_golden as tog
    return tog.sac_noise(meta, g)


def _gpu_errors(meta, g, tr, use_device_batch=False):
    errs = {}
    for s in range(meta["steps"]):
        idx = g[f"s{s}/idx"]
        if use_device_batch:
            raise NotImplementedError
        tr.end_epoch(s)
        tr.train_from_torch(batch_from(meta, idx), eps1=g[f"s{s}/eps1"], eps2=g[f"s{s}/eps2"])
        torch.cuda.synchronize()
        for grp, mod, order in (("policy", tr.policy, PARAM_ORDER_POLICY),
                                ("qf1", tr.qf1, PARAM_ORDER_Q), ("qf2", tr.qf2, PARAM_ORDER_Q)):
            gv = module_tensors(tr, mod, tr.grads)
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, gv[pn].cpu().numpy())
        if meta["auto_alpha"]:
            a = tr.alpha_state.cpu().numpy()
            errs[f"s{s}/grad/log_alpha"] = parity.rel_err(a[5:6], g[f"s{s}/grad/log_alpha"])
            errs[f"s{s}/post/log_alpha"] = parity.rel_err(a[0:1], g[f"s{s}/post/log_alpha"])
        for grp, mod in (("policy", tr.policy), ("qf1", tr.qf1), ("qf2", tr.qf2),
                         ("target_qf1", tr.target_qf1), ("target_qf2", tr.target_qf2)):
            for pn, t in mod.state_dict().items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp in ("policy", "qf1", "qf2") else None
                errs[key], _ = parity.compare_post(g, key, gk, t.cpu().numpy(), meta["lr"])
        st = tr.get_diagnostics()
        for k in ("QF1 Loss", "QF2 Loss", "Q Loss", "Policy Loss", "Alpha", "Alpha Loss",
                  "QF mean", "Log Pis Mean", "Q Targets Mean", "Policy log std Mean"):
            if f"s{s}/stat/{k}" in g:
                errs[f"s{s}/stat/{k}"] = parity.stat_err(st[k], g, f"s{s}/stat/{k}")
    return errs


@pytest.mark.parametrize("name", SAC_FIXTURES)
def test_sac_step_matches_reference_golden(name):
    meta, g = parity.load(name)
    tr = sac_trainer_for(meta)
    errs = _gpu_errors(meta, g, tr)
    noise = _oracle_noise(meta, g)
    bad = {k: (v, noise.get(k, 0.0)) for k, v in errs.items()
           if v > parity.gate(k, noise.get(k, 0.0))}
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
    print(name, "worst", worst)
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def test_stats_keys_match_reference_order():
    meta, g = parity.load("sac_small")
    tr = sac_trainer_for(meta)
    tr.train_from_torch(batch_from(meta, g["s0/idx"]), eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    keys = [k[len("s0/stat/"):] for k in g if k.startswith("s0/stat/")]
    assert list(tr.get_diagnostics().keys()) == keys


def test_graph_replay_is_bitwise_equal_to_direct_launches():
    meta, g = parity.load("sac_small")
    outs = []
    for use_graph in (False, True):
        tr = sac_trainer_for(meta, use_graph=use_graph)
        for s in range(meta["steps"]):
            tr.train_from_torch(batch_from(meta, g[f"s{s}/idx"]), eps1=g[f"s{s}/eps1"],
                                eps2=g[f"s{s}/eps2"])
        outs.append(torch.cat([tr.params, tr.targets, tr.adam_m, tr.adam_v, tr.alpha_state]).cpu())
    assert torch.equal(outs[0], outs[1])


def test_large_batch_graph_replay_with_device_records_is_bitwise():
    """B=4096 (the large-batch kernels, whose GemmBatch records live in device
    memory once a plan has launched them, kernels.h BatchCache): direct
    launches; a graph captured after direct steps filled the cache (the
    captured launches keep the device records' pointers); a graph captured on
    the first call (nothing cached, nothing uploaded under capture: by-value
    records) -- all three bitwise equal."""
    meta, g = parity.load("sac_humanoid_b4096")
    n = min(3, meta["steps"])
    outs = []
    for mode in ("direct", "graph_after_direct", "graph_first"):
        tr = sac_trainer_for(meta, use_graph=(mode == "graph_first"))
        for s in range(n):
            if mode == "graph_after_direct" and s == 1:
                tr.use_graph = True
            tr.train_from_torch(batch_from(meta, g[f"s{s}/idx"]), eps1=g[f"s{s}/eps1"],
                                eps2=g[f"s{s}/eps2"])
        outs.append(torch.cat([tr.params, tr.targets, tr.adam_m, tr.adam_v, tr.alpha_state]).cpu())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])


def test_device_gather_step_equals_host_batch_step():
    """ReplayBuffer.random_batch -> DeviceBatch -> in-step gather gives the
    same result as the reference-format numpy batch."""
    from oac_amd import ReplayBuffer
    meta, g = parity.load("sac_small")
    tr_a = sac_trainer_for(meta)
    tr_b = sac_trainer_for(meta)
    data = synthetic_transitions(meta["n_replay"], meta["obs_dim"], meta["act_dim"], seed=0)
    rb = ReplayBuffer(meta["n_replay"], meta["obs_dim"], meta["act_dim"])
    rb.add_path(dict(data, agent_infos=None, env_infos=None))
    np.random.seed(meta["idx_seed"])
    for s in range(meta["steps"]):
        db = rb.random_batch(meta["B"])
        assert np.array_equal(db.indices.cpu().numpy(), g[f"s{s}/idx"])
        # materialised fields equal the reference's gather + fp32 cast
        assert np.array_equal(db["observations"].cpu().numpy(),
                              data["observations"][g[f"s{s}/idx"]].astype(np.float32))
        tr_a.train_device_batch(db, eps1=g[f"s{s}/eps1"], eps2=g[f"s{s}/eps2"])
        tr_b.train_from_torch(batch_from(meta, g[f"s{s}/idx"]), eps1=g[f"s{s}/eps1"],
                              eps2=g[f"s{s}/eps2"])
    assert torch.equal(tr_a.params, tr_b.params)
    assert torch.equal(tr_a.targets, tr_b.targets)


def test_device_randint_matches_numpy_golden():
    from oac_amd import ReplayBuffer
    meta, g = parity.load("randint")
    rb = ReplayBuffer(4, 3, 2)
    for c in range(meta["n_cases"]):
        seed, size, B = int(g[f"c{c}/seed"]), int(g[f"c{c}/size"]), int(g[f"c{c}/B"])
        rb.seed_device_stream(seed)
        got = []
        for n, cnt in ((size, B), (size, B), (1, 7), (size, B)):
            rb._size = n
            got.append(rb.sample_indices_device(cnt).cpu().numpy().astype(np.int64)
                       & 0xffffffff)
        assert np.array_equal(np.concatenate(got), g[f"c{c}/idx"]), (seed, size, B)


def test_device_randint_long_stream():
    """Many twists: 200k draws at size 1e6 equal numpy's stream."""
    from oac_amd import ReplayBuffer
    rb = ReplayBuffer(4, 3, 2)
    rb.seed_device_stream(12345)
    rb._size = 1_000_000
    got = np.concatenate([rb.sample_indices_device(4096).cpu().numpy() for _ in range(50)])
    np.random.seed(12345)
    ref = np.concatenate([np.random.randint(0, 1_000_000, 4096) for _ in range(50)])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("name", ["oac_expl_humanoid", "oac_expl_small"])
def test_oac_exploration_matches_reference_golden(name):
    from oac_amd import get_optimistic_exploration_action
    meta, g = parity.load(name)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    m = dict(obs_dim=meta["obs_dim"], act_dim=meta["act_dim"], hidden=meta["hidden"],
             discount=0.99, reward_scale=1.0, lr=3e-4, tau=5e-3, auto_alpha=True, log_alpha0=0.0,
             seed=meta["seed"], pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    tr = sac_trainer_for(m, params=params)
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=False)
    for i in range(meta["n_obs"]):
        a, info = get_optimistic_exploration_action(g["obs"][i], policy=tr.policy, qfs=tr.qfs,
                                                    hyper_params=hp, eps=g["eps"][i],
                                                    return_info=True)
        assert a.dtype == np.float32 and a.shape == (meta["act_dim"],)
        assert parity.rel_err(info["std"], g["std"][i]) <= 1e-5
        assert parity.rel_err(info["mu_E"], g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(a, g["action"][i]) <= parity.TOL


@pytest.mark.parametrize("name", ["oac_expl_humanoid", "oac_expl_small"])
def test_batched_oac_exploration_equals_single_calls(name):
    """Vectorised rollouts: all n_obs observations in one call match the
    reference golden and are bitwise the single-observation calls."""
    from oac_amd import get_optimistic_exploration_action, get_optimistic_exploration_actions
    meta, g = parity.load(name)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    m = dict(obs_dim=meta["obs_dim"], act_dim=meta["act_dim"], hidden=meta["hidden"],
             discount=0.99, reward_scale=1.0, lr=3e-4, tau=5e-3, auto_alpha=True, log_alpha0=0.0,
             seed=meta["seed"], pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    tr = sac_trainer_for(m, params=params)
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=False)
    A, info = get_optimistic_exploration_actions(g["obs"], policy=tr.policy, qfs=tr.qfs,
                                                 hyper_params=hp, eps=g["eps"], return_info=True)
    assert A.shape == (meta["n_obs"], meta["act_dim"]) and A.dtype == np.float32
    for i in range(meta["n_obs"]):
        assert parity.rel_err(A[i], g["action"][i]) <= parity.TOL
        assert parity.rel_err(info["mu_E"][i], g["mu_E"][i]) <= parity.TOL
        a, _ = get_optimistic_exploration_action(g["obs"][i], policy=tr.policy, qfs=tr.qfs,
                                                 hyper_params=hp, eps=g["eps"][i])
        np.testing.assert_array_equal(a, A[i])
    # Philox path: finite, in (-1, 1), distinct rows, counter advanced once per call
    c0 = int(tr.step_state[2].item())
    A2, _ = get_optimistic_exploration_actions(g["obs"], policy=tr.policy, qfs=tr.qfs,
                                               hyper_params=hp)
    assert np.isfinite(A2).all() and np.abs(A2).max() < 1
    assert int(tr.step_state[2].item()) == c0 + 1


@pytest.mark.parametrize("n", [64, 300])
def test_exploration_group_sizes_and_paths_bitwise(n):
    """The split kernel's group size follows the observations per launch (16
    workgroups per row at 1..16 rows, 4 at 64, 1 at >= 256 -- then two launches
    for 300 rows) and its hand-off form with it; every row is bitwise the
    single-observation call, the golden rows stay within tolerance, and the
    captured-graph path (oac_expl_action) equals the direct one."""
    from oac_amd import get_optimistic_exploration_action, get_optimistic_exploration_actions
    from oac_amd import optimistic_exploration as oe
    meta, g = parity.load("oac_expl_humanoid")
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    m = dict(obs_dim=meta["obs_dim"], act_dim=meta["act_dim"], hidden=meta["hidden"],
             discount=0.99, reward_scale=1.0, lr=3e-4, tau=5e-3, auto_alpha=True, log_alpha0=0.0,
             seed=meta["seed"], pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    tr = sac_trainer_for(m, params=params)
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=False)
    k = meta["n_obs"]
    rs = np.random.RandomState(n)
    obs = np.concatenate([g["obs"], rs.standard_normal((n - k, meta["obs_dim"]))])
    eps = np.concatenate([g["eps"], rs.standard_normal((n - k, meta["act_dim"]))]).astype(np.float32)
    A, info = get_optimistic_exploration_actions(obs, policy=tr.policy, qfs=tr.qfs,
                                                 hyper_params=hp, eps=eps, return_info=True)
    assert np.isfinite(A).all()
    for i in range(k):
        assert parity.rel_err(A[i], g["action"][i]) <= parity.TOL
        assert parity.rel_err(info["mu_E"][i], g["mu_E"][i]) <= parity.TOL
    for i in sorted({0, 1, k, n // 2, 255 % n, min(256, n - 1), n - 1}):
        a, _ = get_optimistic_exploration_action(obs[i], policy=tr.policy, qfs=tr.qfs,
                                                 hyper_params=hp, eps=eps[i])
        np.testing.assert_array_equal(a, A[i])
    oe._USE_GRAPH = True
    try:
        Ag, _ = get_optimistic_exploration_actions(obs, policy=tr.policy, qfs=tr.qfs,
                                                   hyper_params=hp, eps=eps)
        a0, _ = get_optimistic_exploration_action(obs[3], policy=tr.policy, qfs=tr.qfs,
                                                  hyper_params=hp, eps=eps[3])
    finally:
        oe._USE_GRAPH = False
    np.testing.assert_array_equal(Ag, A)
    np.testing.assert_array_equal(a0, A[3])
    c0 = int(tr.step_state[2].item())
    A2, _ = get_optimistic_exploration_actions(obs, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    assert np.isfinite(A2).all() and np.abs(A2).max() <= 1   # random rows may saturate tanh
    assert not np.array_equal(A2, A)
    assert int(tr.step_state[2].item()) == c0 + 1


@pytest.mark.parametrize("name", ["oac_expl_shared_ant", "oac_expl_shared_small"])
def test_oac_exploration_shared_matches_reference_golden(name):
    """One shared-layer critic with K heads (ParticleTrainerOAC, share_layers):
    single calls against the reference golden, the batched call bitwise equal
    to the single calls."""
    from oac_amd import (ParticleTrainerOAC, get_optimistic_exploration_action,
                         get_optimistic_exploration_actions)
    from gpu_helpers import Space, producers
    meta, g = parity.load(name)
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"], q_out=K,
                        q_last_bias=np.linspace(0.0, 50.0, K))
    pp, qp = producers(params, q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                       "target_qf1"))
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(meta["act_dim"]),
                            deterministic=False, q_min=0.0, q_max=50.0, share_layers=True)
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=True)
    A, _ = get_optimistic_exploration_actions(g["obs"], policy=tr.policy, qfs=tr.qfs,
                                              hyper_params=hp, eps=g["eps"])
    for i in range(meta["n_obs"]):
        a, info = get_optimistic_exploration_action(g["obs"][i], policy=tr.policy, qfs=tr.qfs,
                                                    hyper_params=hp, eps=g["eps"][i],
                                                    return_info=True)
        assert parity.rel_err(info["std"], g["std"][i]) <= 1e-5
        assert parity.rel_err(info["mu_E"], g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(a, g["action"][i]) <= parity.TOL
        np.testing.assert_array_equal(a, A[i])
    with pytest.raises(ValueError):
        get_optimistic_exploration_action(g["obs"][0], policy=tr.policy, qfs=tr.qfs,
                                          hyper_params=dict(hp, share_layers=False))


@pytest.mark.parametrize("name", ["oac_expl_ub_ant", "oac_expl_ub_small"])
def test_oac_exploration_trainer_ub_matches_reference_golden(name):
    """--trainer_UB with the P-OAC ParticleTrainer (particle_trainer_oac.py:147-167):
    Q_UB = the head sorted at delta_index.  Single calls against the reference
    golden, the batched call bitwise equal to them, and the qfs-only call of the
    same handle switching back to mean + beta std."""
    from oac_amd import (ParticleTrainerOAC, get_optimistic_exploration_action,
                         get_optimistic_exploration_actions)
    from gpu_helpers import Space, producers
    meta, g = parity.load(name)
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"], q_out=K,
                        q_last_bias=np.linspace(0.0, 50.0, K))
    pp, qp = producers(params, q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                       "target_qf1"))
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(meta["act_dim"]),
                            deterministic=False, q_min=0.0, q_max=50.0, share_layers=True,
                            delta=meta["ub_delta"])
    assert tr.delta_index == meta["delta_index"]
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=True)
    A, _ = get_optimistic_exploration_actions(g["obs"], policy=tr.policy, qfs=tr.qfs, trainer=tr,
                                              hyper_params=hp, eps=g["eps"])
    for i in range(meta["n_obs"]):
        a, info = get_optimistic_exploration_action(g["obs"][i], policy=tr.policy, qfs=tr.qfs,
                                                    trainer=tr, hyper_params=hp, eps=g["eps"][i],
                                                    return_info=True)
        assert parity.rel_err(info["std"], g["std"][i]) <= 1e-5
        assert parity.rel_err(info["mu_E"], g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(a, g["action"][i]) <= parity.TOL
        np.testing.assert_array_equal(a, A[i])
    # the same handle without trainer: the mean + beta std bound again (oracle)
    P = so.to_torch_params(params["policy"])
    Q = so.to_torch_params(params["qf1"])
    a, _ = get_optimistic_exploration_action(g["obs"][0], policy=tr.policy, qfs=tr.qfs,
                                             hyper_params=hp, eps=g["eps"][0])
    r = so.oac_exploration_action_shared(g["obs"][0], P, Q, meta["beta_UB"], meta["delta"],
                                         g["eps_discard"][0], g["eps"][0])
    assert parity.rel_err(a, r["action"].numpy()) <= parity.TOL


def test_single_call_philox_path():
    """The per-environment-step production path (path_collector.py:219-220):
    an eps-free single call goes through _action_now (cached owner check, the
    observation in the kernel arguments, tagged output granules, the Philox
    draw and the expl_counter advance by the last arrival).  Two calls on one
    observation differ, each advances step_state[2] by exactly 1, and the
    first equals row 0 of an N=1 batched Philox call at the same counter."""
    from oac_amd import get_optimistic_exploration_action, get_optimistic_exploration_actions
    meta, g = parity.load("oac_expl_humanoid")
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    m = dict(obs_dim=meta["obs_dim"], act_dim=meta["act_dim"], hidden=meta["hidden"],
             discount=0.99, reward_scale=1.0, lr=3e-4, tau=5e-3, auto_alpha=True, log_alpha0=0.0,
             seed=meta["seed"], pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    tr = sac_trainer_for(m, params=params)
    hp = dict(beta_UB=meta["beta_UB"], delta=meta["delta"], share_layers=False)
    ob = g["obs"][0]
    c0 = int(tr.step_state[2].item())
    a1, info = get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    assert info == {}
    assert int(tr.step_state[2].item()) == c0 + 1
    a2, _ = get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    assert int(tr.step_state[2].item()) == c0 + 2
    assert a1.shape == (meta["act_dim"],) and a1.dtype == np.float32
    assert np.isfinite(a1).all() and not np.array_equal(a1, a2)
    tr.step_state[2] = c0   # the same counter again, through the batched call
    A, _ = get_optimistic_exploration_actions(ob[None, :], policy=tr.policy, qfs=tr.qfs,
                                              hyper_params=hp)
    np.testing.assert_array_equal(A[0], a1)
    assert int(tr.step_state[2].item()) == c0 + 1
    # the cached validation still rejects a foreign critic list
    with pytest.raises(NotImplementedError):
        get_optimistic_exploration_action(ob, policy=tr.policy, qfs=[tr.qf2, tr.qf1],
                                          hyper_params=hp)
