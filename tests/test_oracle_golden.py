"""Pin the CPU oracle (oracle/) against golden vectors produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from fixtures_lib import (goac_params, ptrain_params, sac_params, synthetic_transitions, PARAM_ORDER_POLICY,
                          PARAM_ORDER_Q)
import parity
from oracle import sac_oracle as so
from oracle.mt_oracle import MT

SAC_FIXTURES = ["sac_small", "sac_stress", "sac_noalpha", "sac_riverswim", "sac_humanoid",
                "sac_humanoid_b4096"]


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
                        log_alpha0=meta["log_alpha0"], dtype=dtype)


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


@pytest.mark.parametrize("name", SAC_FIXTURES)
def test_sac_oracle_matches_reference_golden(name):
    meta, g = parity.load(name)
    errs = sac_errors(meta, g, make_sac_oracle(meta))
    noise = sac_errors(meta, g, make_sac_oracle(meta, torch.float64))
    bad = {k: (v, noise[k]) for k, v in errs.items() if v > parity.gate(k, noise[k])}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def test_poac_oracle_matches_reference_golden():
    for name in ("poac_small", "poac_ant", "poac_counts", "poac_nobias"):
        meta, g = parity.load(name)
        params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                            q_out=meta["K"], q_last_bias=np.linspace(meta["q_min"], meta["q_max"],
                                                                      meta["K"]),
                            pi_init_w=meta["pi_init_w"])
        orc = so.ParticleOACOracle(params, meta["obs_dim"], meta["act_dim"], meta["K"],
                                   discount=meta["discount"], policy_lr=meta["lr"],
                                   qf_lr=meta["lr"], tau=meta["tau"],
                                   train_bias=meta.get("train_bias", True))
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
            for grp, params_ in (("policy", orc.P), ("qf", orc.Q), ("tf", orc.T)):
                for pn, t in params_.items():
                    key = f"s{s}/post/{grp}/{pn}"
                    gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                    errs[key], _ = parity.compare_post(g, key, gk, t.numpy(), meta["lr"])
            for i in range(meta["K"]):
                k = f"s{s}/stat/QF{i} Loss"
                errs[k] = parity.rel_err(out["qf_losses"][i].item(), g[k])
        bad = {k: v for k, v in errs.items()
               if v > (parity.TOL if k.startswith("s0/") else 1e-4)}
        assert not bad, (name, sorted(bad.items(), key=lambda kv: -kv[1])[:10])


GOAC_FIXTURES = ["goac_small", "goac_counts", "goac_soft", "goac_humanoid", "goac_nobias"]
GOAC_STATS = ("QF mean", "QF std", "QF Loss", "STD Loss", "Q Target Mean", "Q STD Target Mean",
              "Policy Loss", "Policy mu Mean", "Policy log std Mean")


def make_goac_oracle(meta, dtype=torch.float32):
    params = goac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                         meta["q_min"], meta["q_max"], pi_init_w=meta["pi_init_w"],
                         q_init_w=meta["q_init_w"])
    return so.GaussianOACOracle(params, meta["obs_dim"], meta["act_dim"], delta=meta["delta"],
                                q_min=meta["q_min"], q_max=meta["q_max"],
                                discount=meta["discount"], policy_lr=meta["lr"],
                                qf_lr=meta["lr"], tau=meta["tau"],
                                std_soft_update_prob=meta["soft"],
                                train_bias=meta.get("train_bias", True), dtype=dtype)


def goac_errors(meta, g, orc):
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
        Da = meta["act_dim"]
        th = out["target_head"]
        st = {"QF mean": out["q_preds"].mean(), "QF std": out["std_preds"].mean(),
              "QF Loss": out["q_loss"], "STD Loss": out["std_loss"],
              "Q Target Mean": out["q_target"].mean(),
              "Q STD Target Mean": out["std_target"].mean(),
              "Policy Loss": out["upper_bound"].mean(), "Policy mu Mean": th["mean"].mean(),
              "Policy log std Mean": th["log_std"].mean()}
        for k in GOAC_STATS:
            errs[f"s{s}/stat/{k}"] = parity.stat_err(float(st[k]), g, f"s{s}/stat/{k}")
    return errs


@pytest.mark.parametrize("name", GOAC_FIXTURES)
def test_goac_oracle_matches_reference_golden(name):
    """GaussianTrainer (g-oac) restatement vs the reference's own run."""
    meta, g = parity.load(name)
    errs = goac_errors(meta, g, make_goac_oracle(meta))
    noise = goac_errors(meta, g, make_goac_oracle(meta, torch.float64))
    bad = {k: (v, noise[k]) for k, v in errs.items() if v > parity.gate(k, noise[k])}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


PTRAIN_FIXTURES = ["ptrain_small", "ptrain_counts", "ptrain_soft_rescale", "ptrain_mean_update",
                   "ptrain_humanoid", "ptrain_nobias"]


def make_ptrain_oracle(meta, dtype=torch.float32):
    params = ptrain_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                           meta["K"], meta["q_min"], meta["q_max"], pi_init_w=meta["pi_init_w"],
                           q_init_w=meta["q_init_w"])
    return so.ParticleUBOracle(params, meta["obs_dim"], meta["act_dim"], meta["K"],
                               meta["delta_index"], q_min=meta["q_min"], q_max=meta["q_max"],
                               discount=meta["discount"], policy_lr=meta["lr"], qf_lr=meta["lr"],
                               tau=meta["tau"], std_soft_update_prob=meta["soft"],
                               mean_update=meta["mean_update"], rescale=meta["rescale"],
                               train_bias=meta.get("train_bias", True), dtype=dtype)


def ptrain_errors(meta, g, orc):
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
        th = out["target_head"]
        st = {"Q Loss": out["qf_loss"], "Policy Loss": out["upper_bound"].mean(),
              "Policy mu Mean": th["mean"].mean(), "Policy log std Mean": th["log_std"].mean(),
              "QF mean": out["sorted_qs"].mean()}
        for i in range(meta["K"]):
            st[f"QF{i} Loss"] = out["qf_losses"][i]
        for k, v in st.items():
            errs[f"s{s}/stat/{k}"] = parity.stat_err(float(v), g, f"s{s}/stat/{k}")
    return errs


@pytest.mark.parametrize("name", PTRAIN_FIXTURES)
def test_ptrain_oracle_matches_reference_golden(name):
    """p-oac ParticleTrainer (particle_trainer.py) restatement vs the
    reference's own run."""
    meta, g = parity.load(name)
    errs = ptrain_errors(meta, g, make_ptrain_oracle(meta))
    noise = ptrain_errors(meta, g, make_ptrain_oracle(meta, torch.float64))
    bad = {k: (v, noise[k]) for k, v in errs.items() if v > parity.gate(k, noise[k])}
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
