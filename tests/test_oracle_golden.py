"""Pin the CPU oracle (oracle/) against golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from fixtures_lib import (goac_params, mid_state, ptrain_params, sac_params, synthetic_transitions, PARAM_ORDER_POLICY,
                          PARAM_ORDER_Q)
import parity
from oracle import sac_oracle as so
from oracle.mt_oracle import MT

SAC_FIXTURES = ["sac_small", "sac_stress", "sac_noalpha", "sac_riverswim", "sac_humanoid",
                "sac_humanoid_b4096", "sac_period2"]


def test_randint_oracle_matches_numpy_golden():
    meta, g = parity.load("randint")
    for c in range(meta["n_cases"]):
        seed, size, B = int(g[f"c{c}/seed"]), int(g[f"c{c}/size"]), int(g[f"c{c}/B"])
        mt = MT(seed)
        got = np.concatenate([mt.randint(size, B), mt.randint(size, B), mt.randint(1, 7),
                              mt.randint(size, B)])
        assert np.array_equal(got, g[f"c{c}/idx"]), (seed, size, B)


def build_batch(meta, idx):
    tr = synthetic_transitions(meta["n_replay"], meta["obs_dim"], meta["act_dim"], seed=0)
    return {k: v[idx] for k, v in tr.items()}


def make_sac_oracle(meta, dtype=torch.float32):
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    return so.SACOracle(params, meta["obs_dim"], meta["act_dim"], discount=meta["discount"],
                        reward_scale=meta["reward_scale"], policy_lr=meta["lr"],
                        qf_lr=meta["lr"], tau=meta["tau"], auto_alpha=meta["auto_alpha"],
                        log_alpha0=meta["log_alpha0"],
                        target_update_period=meta.get("target_update_period", 1), dtype=dtype)


def sac_errors(meta, g, orc, steps=None):
    """Run the oracle through the fixture's steps; return {key: err}."""
    errs = {}
    for s in range(steps or meta["steps"]):
        batch = build_batch(meta, g[f"s{s}/idx"])
        out = orc.step(batch, g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp, order in (("policy", PARAM_ORDER_POLICY), ("qf1", PARAM_ORDER_Q),
                           ("qf2", PARAM_ORDER_Q)):
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, out["grads"][grp][pn].numpy())
        if meta["auto_alpha"]:
            errs[f"s{s}/grad/log_alpha"] = parity.rel_err(out["grads"]["log_alpha"].numpy(),
                                                          g[f"s{s}/grad/log_alpha"])
            errs[f"s{s}/post/log_alpha"] = parity.rel_err(orc.log_alpha.numpy(),
                                                          g[f"s{s}/post/log_alpha"])
        for grp, params in (("policy", orc.P), ("qf1", orc.Q1), ("qf2", orc.Q2),
                            ("target_qf1", orc.T1), ("target_qf2", orc.T2)):
            for pn, t in params.items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp in ("policy", "qf1", "qf2") else None
                e, _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
                errs[key] = e
        st = out["stats"]
        for k in ("QF1 Loss", "QF2 Loss", "Q Loss", "Policy Loss", "Alpha", "Alpha Loss",
                  "QF mean", "Log Pis Mean", "Q Targets Mean", "Policy log std Mean"):
            if f"s{s}/stat/{k}" in g:
                errs[f"s{s}/stat/{k}"] = parity.stat_err(st[k], g, f"s{s}/stat/{k}")
    return errs


def _inputs_of(g):
    return {k: v for k, v in g.items() if k.split("/")[-1] in ("idx", "eps1", "eps2", "counts")}


def sac_record(meta, g, orc):
    """A run of ``orc`` through the fixture's inputs, keyed like the fixture
    (every tensor whole): a stand-in golden for the spread measurement."""
    rec = _inputs_of(g)
    for s in range(meta["steps"]):
        out = orc.step(build_batch(meta, g[f"s{s}/idx"]), g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp in ("policy", "qf1", "qf2"):
            for pn, t in out["grads"][grp].items():
                rec[f"s{s}/grad/{grp}/{pn}"] = t.numpy().copy()
        if meta["auto_alpha"]:
            rec[f"s{s}/grad/log_alpha"] = out["grads"]["log_alpha"].numpy().copy()
            rec[f"s{s}/post/log_alpha"] = orc.log_alpha.numpy().copy()
        for grp, params in (("policy", orc.P), ("qf1", orc.Q1), ("qf2", orc.Q2),
                            ("target_qf1", orc.T1), ("target_qf2", orc.T2)):
            for pn, t in params.items():
                rec[f"s{s}/post/{grp}/{pn}"] = t.numpy().copy()
        for k, v in out["stats"].items():
            rec[f"s{s}/stat/{k}"] = np.array(v, np.float64)
    return rec


def noise_of(errors_fn, record_fn, make_fn, meta, g):
    """Per-key fp32 noise for the trajectory gate (parity.gate): the larger of
    the reference's own distance from the float64 oracle and an fp32
    oracle run's distance from the same float64 run.  Both are correct fp32
    evaluations; past step 0 their trajectories part by what the rounding of
    Adam's lr * sign(g) band and of ReLU masks near 0 does, which a single
    float64 comparison of the reference can understate by orders of magnitude
    (sac_humanoid_b4096 step 2: the reference sits 9e-7 from float64 on the
    policy fc0 gradient, an fp32 oracle run 5e-4).  The per-step check at
    1e-5 is the teacher-forced one (test_gpu_teacher.py) and the mid-state
    fixtures (test_*_mid_state_*)."""
    ref = errors_fn(meta, g, make_fn(meta, torch.float64))
    rec64 = record_fn(meta, g, make_fn(meta, torch.float64))
    spread = errors_fn(meta, rec64, make_fn(meta))
    # step 0 has no trajectory to part along: its gate stays the reference's
    # own distance from float64 (1e-5 unless the reference itself is further
    # off, as in the saturated-tanh stress fixture), for every fixture
    return {k: v if k.startswith("s0/") else max(v, spread.get(k, 0.0)) for k, v in ref.items()}


def sac_noise(meta, g):
    return noise_of(sac_errors, sac_record, make_sac_oracle, meta, g)


@pytest.mark.parametrize("name", SAC_FIXTURES)
def test_sac_oracle_matches_reference_golden(name):
    meta, g = parity.load(name)
    errs = sac_errors(meta, g, make_sac_oracle(meta))
    noise = sac_noise(meta, g)
    bad = {k: (v, noise[k]) for k, v in errs.items() if v > parity.gate(k, noise[k])}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def load_mid_state(orc, tr_groups, meta, params):
    """Put fixtures_lib.mid_state (the mid-state goldens' starting point)
    into an oracle: Adam moments and step count, log-alpha and its moments."""
    ms = mid_state(params, [p for p, _ in tr_groups], meta["mid_state"]["t"],
                   meta["mid_state"]["seed"])
    for grp, opt in tr_groups:
        for pn, (m, v) in ms[grp].items():
            opt.m[pn].copy_(torch.from_numpy(m).to(opt.m[pn].dtype))
            opt.v[pn].copy_(torch.from_numpy(v).to(opt.v[pn].dtype))
        opt.t = ms["t"]
    orc.log_alpha.fill_(float(ms["log_alpha"]))
    am, av = ms["alpha_adam"]
    orc.opt_a.m["log_alpha"].fill_(float(am))
    orc.opt_a.v["log_alpha"].fill_(float(av))
    orc.opt_a.t = ms["t"]
    orc.n_steps = ms["t"]
    return ms


def adam_errors(g, s, opts):
    """Post-step Adam moments (sampled in the mid-state fixtures)."""
    errs = {}
    for grp, opt in opts:
        for pn in opt.m:
            for nm, t in (("exp_avg", opt.m[pn]), ("exp_avg_sq", opt.v[pn])):
                key = f"s{s}/adam/{grp}/{pn}/{nm}"
                if parity.has(g, key):
                    errs[key] = parity.compare(g, key, t.numpy())
    return errs


def make_sac_mid_oracle(meta, dtype=torch.float32):
    orc = make_sac_oracle(meta, dtype)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    load_mid_state(orc, [("policy", orc.opt_p), ("qf1", orc.opt_q1), ("qf2", orc.opt_q2)],
                   meta, params)
    return orc


@pytest.mark.parametrize("name", ["sac_humanoid_mid", "sac_humanoid_b4096_mid"])
def test_sac_oracle_mid_state_step_matches_reference(name):
    """One step from a mid-training state (Adam moments after t = 7 steps,
    log-alpha off its init) at the BASELINE dims: every gradient (whole),
    sampled post-step parameters / targets / Adam moments, log-alpha and the
    losses against the reference at 1e-5 -- the per-step pin of what steps
    past the first add (trainer/trainer.py:139-224, torch-1.4 Adam)."""
    meta, g = parity.load(name)
    orc = make_sac_mid_oracle(meta)
    errs = sac_errors(meta, g, orc)
    errs.update(adam_errors(g, 0, [("policy", orc.opt_p), ("qf1", orc.opt_q1),
                                   ("qf2", orc.opt_q2)]))
    noise = sac_errors(meta, g, make_sac_mid_oracle(meta, torch.float64))
    bad = {k: (v, noise.get(k)) for k, v in errs.items() if v > parity.TOL}
    print(name, sorted(errs.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def stats_of(name, x):
    """create_stats_ordered_dict (utils/eval_util.py:70-110): Mean, Std
    (population), Max, Min of an array."""
    x = np.asarray(x.detach().numpy() if torch.is_tensor(x) else x, np.float64)
    return {f"{name} Mean": x.mean(), f"{name} Std": x.std(), f"{name} Max": x.max(),
            f"{name} Min": x.min()}


# integer counts of the sorted heads (exact on both sides; not a float statistic)
COUNT_STATS = ("QF Unordered", "QF target Undordered")


def stat_errors(s, g, st):
    """{key: err} for every float statistic of step s the fixture holds."""
    errs = {}
    for k in g:
        if not k.startswith(f"s{s}/stat/"):
            continue
        name = k[len(f"s{s}/stat/"):]
        if name in COUNT_STATS:
            continue
        assert name in st, (k, "statistic not restated by the oracle")
        errs[k] = parity.stat_err(float(st[name]), g, k)
    return errs


POAC_FIXTURES = ["poac_small", "poac_ant", "poac_ant_b4096", "poac_counts", "poac_nobias",
                 "poac_period2"]


def make_poac_oracle(meta, dtype=torch.float32):
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        q_out=meta["K"], q_last_bias=np.linspace(meta["q_min"], meta["q_max"],
                                                                  meta["K"]),
                        pi_init_w=meta["pi_init_w"])
    return so.ParticleOACOracle(params, meta["obs_dim"], meta["act_dim"], meta["K"],
                                discount=meta["discount"], policy_lr=meta["lr"],
                                qf_lr=meta["lr"], tau=meta["tau"],
                                target_update_period=meta.get("target_update_period", 1),
                                train_bias=meta.get("train_bias", True), dtype=dtype)


def poac_stats(meta, out):
    """particle_trainer_oac.py:335-362."""
    qs = out["sorted_qs"].detach().numpy().astype(np.float64)
    st = {"QF mean": np.mean(qs, axis=0).mean(), "QF std": np.std(qs, axis=0).mean()}
    for i in range(meta["K"]):
        st[f"QF{i} Loss"] = float(out["qf_losses"][i])
        st.update(stats_of(f"Q{i}Predictions", out["sorted_qs"][i]))
        st.update(stats_of(f"Q{i}Targets", out["tq"][i]))
    st["Policy Loss"] = float(out["policy_loss"])
    st.update(stats_of("Policy mu", out["policy_mean"]))
    st.update(stats_of("Policy log std", out["policy_log_std"]))
    return st


def poac_errors(meta, g, orc):
    """Run the P-OAC oracle through the fixture's steps; return {key: err}
    over gradients, log-alpha, post-step parameters and statistics."""
    errs = {}
    for s in range(meta["steps"]):
        b = build_batch(meta, g[f"s{s}/idx"])
        if meta.get("counts"):
            b["counts"] = g[f"s{s}/counts"][:, None]
        out = orc.step(b, g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp, order in (("policy", PARAM_ORDER_POLICY), ("qf", PARAM_ORDER_Q)):
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, out["grads"][grp][pn].numpy())
        errs[f"s{s}/grad/log_alpha"] = parity.rel_err(out["grads"]["log_alpha"].numpy(),
                                                      g[f"s{s}/grad/log_alpha"])
        errs[f"s{s}/post/log_alpha"] = parity.rel_err(orc.log_alpha.numpy(),
                                                      g[f"s{s}/post/log_alpha"])
        for grp, params_ in (("policy", orc.P), ("qf", orc.Q), ("tf", orc.T)):
            for pn, t in params_.items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
        errs.update(stat_errors(s, g, poac_stats(meta, out)))
    return errs


def gated(errs, noise):
    """The keys whose error exceeds the noise-derived gate (parity.gate)."""
    return {k: (v, noise.get(k, 0.0)) for k, v in errs.items()
            if v > parity.gate(k, noise.get(k, 0.0))}


def poac_record(meta, g, orc):
    rec = _inputs_of(g)
    for s in range(meta["steps"]):
        b = build_batch(meta, g[f"s{s}/idx"])
        if meta.get("counts"):
            b["counts"] = g[f"s{s}/counts"][:, None]
        out = orc.step(b, g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp in ("policy", "qf"):
            for pn, t in out["grads"][grp].items():
                rec[f"s{s}/grad/{grp}/{pn}"] = t.numpy().copy()
        rec[f"s{s}/grad/log_alpha"] = out["grads"]["log_alpha"].numpy().copy()
        rec[f"s{s}/post/log_alpha"] = orc.log_alpha.numpy().copy()
        for grp, params_ in (("policy", orc.P), ("qf", orc.Q), ("tf", orc.T)):
            for pn, t in params_.items():
                rec[f"s{s}/post/{grp}/{pn}"] = t.numpy().copy()
        for k, v in poac_stats(meta, out).items():
            rec[f"s{s}/stat/{k}"] = np.array(v, np.float64)
        for k in COUNT_STATS:
            if f"s{s}/stat/{k}" in g:
                rec[f"s{s}/stat/{k}"] = g[f"s{s}/stat/{k}"]
    return rec


def poac_noise(meta, g):
    return noise_of(poac_errors, poac_record, make_poac_oracle, meta, g)


@pytest.mark.parametrize("name", POAC_FIXTURES)
def test_poac_oracle_matches_reference_golden(name):
    """particle_trainer_oac.ParticleTrainer restatement vs the reference's own
    run, every step under the noise-derived gate (noise_of)."""
    meta, g = parity.load(name)
    errs = poac_errors(meta, g, make_poac_oracle(meta))
    bad = gated(errs, poac_noise(meta, g))
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def make_poac_mid_oracle(meta, dtype=torch.float32):
    orc = make_poac_oracle(meta, dtype)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        q_out=meta["K"], q_last_bias=np.linspace(meta["q_min"], meta["q_max"],
                                                                 meta["K"]),
                        pi_init_w=meta["pi_init_w"])
    load_mid_state(orc, [("policy", orc.opt_p), ("qf1", orc.opt_q)], meta, params)
    return orc


def test_poac_oracle_mid_state_step_matches_reference():
    """BASELINE configs[4] (K=10, Ant-v2 dims, B=4096): one step from a
    mid-training state against the reference at 1e-5
    (trainer/particle_trainer_oac.py:169-363)."""
    meta, g = parity.load("poac_ant_b4096_mid")
    orc = make_poac_mid_oracle(meta)
    errs = poac_errors(meta, g, orc)
    errs.update(adam_errors(g, 0, [("policy", orc.opt_p), ("qf", orc.opt_q)]))
    bad = {k: v for k, v in errs.items() if v > parity.TOL}
    print(sorted(errs.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1])[:10]


GOAC_FIXTURES = ["goac_small", "goac_counts", "goac_soft", "goac_humanoid", "goac_nobias",
                 "goac_tpn"]


def next_policy_of(g):
    """use_target_policy fixtures: the DDPG target network's weights."""
    tpn = {k[4:]: v for k, v in g.items() if k.startswith("tpn/")}
    return tpn or None


def make_goac_oracle(meta, dtype=torch.float32, g=None):
    params = goac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                         meta["q_min"], meta["q_max"], pi_init_w=meta["pi_init_w"],
                         q_init_w=meta["q_init_w"])
    return so.GaussianOACOracle(params, meta["obs_dim"], meta["act_dim"], delta=meta["delta"],
                                q_min=meta["q_min"], q_max=meta["q_max"],
                                discount=meta["discount"], policy_lr=meta["lr"],
                                qf_lr=meta["lr"], tau=meta["tau"],
                                std_soft_update_prob=meta["soft"],
                                train_bias=meta.get("train_bias", True),
                                next_policy=next_policy_of(g) if g is not None else None,
                                dtype=dtype)


def goac_stats(out):
    """gaussian_trainer.py:400-436 ('Policy mu / log std' describe the target
    policy: the variable is reassigned by its forward)."""
    st = {"QF mean": float(out["q_preds"].mean()), "QF std": float(out["std_preds"].mean()),
          "QF Loss": float(out["q_loss"])}
    st.update(stats_of("Q Predictions", out["q_preds"]))
    st.update(stats_of("Q Target", out["q_target"]))
    st["STD Loss"] = float(out["std_loss"])
    st.update(stats_of("Q STD Predictions", out["std_preds"]))
    st.update(stats_of("Q STD Target", out["std_target"]))
    st["Policy Loss"] = float(out["upper_bound"].mean())
    st.update(stats_of("Policy mu", out["target_head"]["mean"]))
    st.update(stats_of("Policy log std", out["target_head"]["log_std"]))
    return st


def det_errors(meta, g, orc, stats_fn):
    errs = {}
    for s in range(meta["steps"]):
        b = build_batch(meta, g[f"s{s}/idx"])
        if meta["counts"]:
            b["counts"] = g[f"s{s}/counts"][:, None]
        out = orc.step(b)
        for grp in ("policy", "target_policy", "qf"):
            for pn in (PARAM_ORDER_Q if grp == "qf" else PARAM_ORDER_POLICY):
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, out["grads"][grp][pn].numpy())
        for grp, params_ in (("policy", orc.P), ("target_policy", orc.TP), ("qf", orc.Q),
                             ("tf", orc.T)):
            for pn, t in params_.items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
        errs.update(stat_errors(s, g, stats_fn(meta, out)))
    return errs


def goac_errors(meta, g, orc):
    return det_errors(meta, g, orc, lambda meta, out: goac_stats(out))


@pytest.mark.parametrize("name", GOAC_FIXTURES)
def test_goac_oracle_matches_reference_golden(name):
    """GaussianTrainer (g-oac) restatement vs the reference's own run."""
    meta, g = parity.load(name)
    errs = goac_errors(meta, g, make_goac_oracle(meta, g=g))
    noise = goac_errors(meta, g, make_goac_oracle(meta, torch.float64, g=g))
    bad = gated(errs, noise)
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


PTRAIN_FIXTURES = ["ptrain_small", "ptrain_counts", "ptrain_soft_rescale", "ptrain_mean_update",
                   "ptrain_humanoid", "ptrain_nobias", "ptrain_tpn"]


def make_ptrain_oracle(meta, dtype=torch.float32, g=None):
    params = ptrain_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                           meta["K"], meta["q_min"], meta["q_max"], pi_init_w=meta["pi_init_w"],
                           q_init_w=meta["q_init_w"])
    return so.ParticleUBOracle(params, meta["obs_dim"], meta["act_dim"], meta["K"],
                               meta["delta_index"], q_min=meta["q_min"], q_max=meta["q_max"],
                               discount=meta["discount"], policy_lr=meta["lr"], qf_lr=meta["lr"],
                               tau=meta["tau"], std_soft_update_prob=meta["soft"],
                               mean_update=meta["mean_update"], rescale=meta["rescale"],
                               train_bias=meta.get("train_bias", True),
                               next_policy=next_policy_of(g) if g is not None else None,
                               dtype=dtype)


def ptrain_stats(meta, out):
    """particle_trainer.py:403-432."""
    qs = out["sorted_qs"].detach().numpy().astype(np.float64)
    st = {"QF mean": np.mean(qs, axis=0).mean(), "QF std": np.std(qs, axis=0).mean(),
          "Q Loss": float(out["qf_loss"])}
    for i in range(meta["K"]):
        st[f"QF{i} Loss"] = float(out["qf_losses"][i])
        st.update(stats_of(f"Q{i}Predictions", out["sorted_qs"][i]))
        st.update(stats_of(f"Q{i}Targets", out["tq"][i]))
    st["Policy Loss"] = float(out["upper_bound"].mean())
    st.update(stats_of("Policy mu", out["target_head"]["mean"]))
    st.update(stats_of("Policy log std", out["target_head"]["log_std"]))
    return st


def ptrain_errors(meta, g, orc):
    return det_errors(meta, g, orc, ptrain_stats)


@pytest.mark.parametrize("name", PTRAIN_FIXTURES)
def test_ptrain_oracle_matches_reference_golden(name):
    """p-oac ParticleTrainer (particle_trainer.py) restatement vs the
    reference's own run."""
    meta, g = parity.load(name)
    errs = ptrain_errors(meta, g, make_ptrain_oracle(meta, g=g))
    noise = ptrain_errors(meta, g, make_ptrain_oracle(meta, torch.float64, g=g))
    bad = gated(errs, noise)
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


@pytest.mark.parametrize("name", ["oac_expl_humanoid", "oac_expl_small"])
def test_oac_exploration_oracle_matches_reference_golden(name):
    meta, g = parity.load(name)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    P = so.to_torch_params(params["policy"])
    Q1 = so.to_torch_params(params["qf1"])
    Q2 = so.to_torch_params(params["qf2"])
    for i in range(meta["n_obs"]):
        r = so.oac_exploration_action(g["obs"][i], P, Q1, Q2, meta["beta_UB"], meta["delta"],
                                      g["eps_discard"][i], g["eps"][i])
        assert parity.rel_err(r["std"].numpy(), g["std"][i]) <= 1e-6
        assert parity.rel_err(r["mu_E"].numpy(), g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(r["action"].numpy(), g["action"][i]) <= parity.TOL


@pytest.mark.parametrize("name", ["oac_expl_shared_ant", "oac_expl_shared_small"])
def test_oac_exploration_shared_oracle_matches_reference_golden(name):
    """K-head (share_layers) OAC shift: the reference's except branch."""
    meta, g = parity.load(name)
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"], q_out=K,
                        q_last_bias=np.linspace(0.0, 50.0, K))
    P = so.to_torch_params(params["policy"])
    Q = so.to_torch_params(params["qf1"])
    for i in range(meta["n_obs"]):
        r = so.oac_exploration_action_shared(g["obs"][i], P, Q, meta["beta_UB"], meta["delta"],
                                             g["eps_discard"][i], g["eps"][i])
        assert parity.rel_err(r["std"].numpy(), g["std"][i]) <= 1e-6
        assert parity.rel_err(r["mu_E"].numpy(), g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(r["action"].numpy(), g["action"][i]) <= parity.TOL


@pytest.mark.parametrize("name", ["oac_expl_ub_ant", "oac_expl_ub_small"])
def test_oac_exploration_trainer_ub_oracle_matches_reference_golden(name):
    """--trainer_UB with particle_trainer_oac.ParticleTrainer: Q_UB =
    trainer.predict = the sorted head delta_index (particle_trainer_oac.py:147-167)."""
    meta, g = parity.load(name)
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"], q_out=K,
                        q_last_bias=np.linspace(0.0, 50.0, K))
    P = so.to_torch_params(params["policy"])
    Q = so.to_torch_params(params["qf1"])
    for i in range(meta["n_obs"]):
        r = so.oac_exploration_action_shared(g["obs"][i], P, Q, meta["beta_UB"], meta["delta"],
                                             g["eps_discard"][i], g["eps"][i],
                                             ub_index=meta["delta_index"])
        assert parity.rel_err(r["std"].numpy(), g["std"][i]) <= 1e-6
        assert parity.rel_err(r["mu_E"].numpy(), g["mu_E"][i]) <= parity.TOL
        assert parity.rel_err(r["action"].numpy(), g["action"][i]) <= parity.TOL


@pytest.mark.parametrize("name", ["sac_small", "sac_stress", "sac_noalpha", "sac_humanoid",
                                  "sac_period2"])
def test_sac_autograd_restatement_matches_reference_golden(name):
    """oracle/sac_autograd.py (the reference's op sequence on torch autograd:
    bench.py's CPU baseline) against the reference's own run: every gradient
    and post-step parameter of every step under the trajectory gate."""
    from oracle.sac_autograd import SACAutograd
    meta, g = parity.load(name)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    ag = SACAutograd(params, meta["obs_dim"], meta["act_dim"], discount=meta["discount"],
                     reward_scale=meta["reward_scale"], policy_lr=meta["lr"], qf_lr=meta["lr"],
                     tau=meta["tau"], auto_alpha=meta["auto_alpha"], log_alpha0=meta["log_alpha0"],
                     target_update_period=meta.get("target_update_period", 1))
    noise = sac_noise(meta, g)
    errs = {}
    for s in range(meta["steps"]):
        out = ag.step(build_batch(meta, g[f"s{s}/idx"]), g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp in ("policy", "qf1", "qf2"):
            for pn, t in out["grads"][grp].items():
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, t.numpy())
        for grp, sd in ag.state().items():
            for pn, t in sd.items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp in ("policy", "qf1", "qf2") else None
                errs[key], _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
        if meta["auto_alpha"]:
            errs[f"s{s}/post/log_alpha"] = parity.rel_err(ag.log_alpha.detach().numpy(),
                                                          g[f"s{s}/post/log_alpha"])
        if f"s{s}/stat/QF1 Loss" in g:
            errs[f"s{s}/stat/QF1 Loss"] = parity.stat_err(float(out["qf1_loss"]), g,
                                                          f"s{s}/stat/QF1 Loss")
    bad = {k: (v, noise.get(k, 0.0)) for k, v in errs.items()
           if v > parity.gate(k, noise.get(k, 0.0))}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


@pytest.mark.parametrize("name", ["poac_small", "poac_ant_b4096", "poac_counts", "poac_period2"])
def test_poac_autograd_restatement_matches_reference_golden(name):
    """oracle/sac_autograd.py ParticleOACAutograd (particle_trainer_oac.py's op
    sequence on torch autograd: bench.py's configs[4] CPU baseline) against
    the reference's own run, every step under the trajectory gate (step 0 at
    the reference's own float64 distance)."""
    from oracle.sac_autograd import ParticleOACAutograd
    meta, g = parity.load(name)
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"], q_out=K,
                        q_last_bias=np.linspace(meta["q_min"], meta["q_max"], K),
                        pi_init_w=meta["pi_init_w"])
    ag = ParticleOACAutograd(params, meta["obs_dim"], meta["act_dim"], K,
                             discount=meta["discount"], policy_lr=meta["lr"], qf_lr=meta["lr"],
                             tau=meta["tau"], target_update_period=meta.get("target_update_period", 1))
    noise = poac_noise(meta, g)
    errs = {}
    for s in range(meta["steps"]):
        b = build_batch(meta, g[f"s{s}/idx"])
        if meta.get("counts"):
            b["counts"] = g[f"s{s}/counts"][:, None]
        out = ag.step(b, g[f"s{s}/eps1"], g[f"s{s}/eps2"])
        for grp in ("policy", "qf"):
            for pn, t in out["grads"][grp].items():
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, t.numpy())
        errs[f"s{s}/grad/log_alpha"] = parity.rel_err(out["grads"]["log_alpha"].numpy(),
                                                      g[f"s{s}/grad/log_alpha"])
        for grp, sd in ag.state().items():
            for pn, t in sd.items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
        for i in range(K):
            if f"s{s}/stat/QF{i} Loss" in g:
                errs[f"s{s}/stat/QF{i} Loss"] = parity.stat_err(float(out["qf_losses"][i]), g,
                                                                f"s{s}/stat/QF{i} Loss")
    bad = gated(errs, noise)
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]
