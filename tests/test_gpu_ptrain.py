"""GPU parity of the p-oac ParticleTrainer of trainer/particle_trainer.py (the
trainer every reproduce_p-oac*.sh recipe runs: share_layers K-particle
critic, deterministic policy, target_policy) against the reference's own
outputs (tests/golden/ptrain_*.npz, make_golden.py gen_ptrain) and, at the
large-batch kernel configuration, against the CPU oracle."""
import numpy as np
import pytest
import torch

import parity
import test_oracle_golden as tog
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q, ptrain_params
from gpu_helpers import Space, StateDictModule, batch_from, module_tensors

pytestmark = pytest.mark.gpu

FIXTURES = ["ptrain_small", "ptrain_counts", "ptrain_soft_rescale", "ptrain_mean_update",
            "ptrain_humanoid", "ptrain_nobias", "ptrain_tpn"]


def ptrain_producers(params):
    """Producers in the reference constructor's call order
    (particle_trainer.py:47-59, 96-106, 141)."""
    # a third policy_producer() call builds use_target_policy's network (its
    # weights are then overwritten: a copy of the policy, then the fixture's)
    pols = iter([params["policy"], params["target_policy"], params["policy"]])
    qs = iter([params["qf1"]] * 4 + [params["qf1"], params["target_qf1"]])
    return (lambda **k: StateDictModule(next(pols)),
            lambda **k: StateDictModule(next(qs)))


def ptrain_trainer_for(meta, params=None, **kw):
    from oac_amd import ParticleTrainer
    if params is None:
        params = ptrain_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                               meta["K"], meta["q_min"], meta["q_max"],
                               pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    pp, qp = ptrain_producers(params)
    soft = meta.get("soft")
    return ParticleTrainer(pp, qp, n_estimators=meta["K"], action_space=Space(meta["act_dim"]),
                           discount=meta["discount"], reward_scale=1.0, delta=meta["delta"],
                           policy_lr=meta["lr"], qf_lr=meta["lr"], soft_target_tau=meta["tau"],
                           target_update_period=1, q_min=meta["q_min"], q_max=meta["q_max"],
                           share_layers=True, counts=bool(meta.get("counts")),
                           mean_update=bool(meta.get("mean_update")),
                           rescale_targets_around_mean=bool(meta.get("rescale")),
                           std_soft_update=soft is not None,
                           std_soft_update_prob=0.0 if soft is None else soft,
                           train_bias=meta.get("train_bias", True),
                           use_target_policy=bool(meta.get("use_target_policy")), **kw)


@pytest.mark.parametrize("name", FIXTURES)
def test_ptrain_step_matches_reference_golden(name):
    meta, g = parity.load(name)
    tr = ptrain_trainer_for(meta)
    if meta.get("use_target_policy"):   # the fixture's DDPG target network weights
        tr.target_policy_network.load_state_dict(
            {k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("tpn/")})
    assert tr.delta_index == meta["delta_index"]
    errs = {}
    for s in range(meta["steps"]):
        tr.end_epoch(s)
        b = batch_from(meta, g[f"s{s}/idx"])
        if meta["counts"]:
            b["counts"] = g[f"s{s}/counts"][:, None]
        tr.train_from_torch(b)
        torch.cuda.synchronize()
        for grp, mod, order in (("policy", tr.policy, PARAM_ORDER_POLICY),
                                ("target_policy", tr.target_policy, PARAM_ORDER_POLICY),
                                ("qf", tr.qfs[0], PARAM_ORDER_Q)):
            gv = module_tensors(tr, mod, tr.grads)
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, gv[pn].cpu().numpy())
        for grp, mod in (("policy", tr.policy), ("target_policy", tr.target_policy),
                         ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
            for pn, t in mod.state_dict().items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.cpu().numpy(), meta["lr"])
        for k, v in tr.get_diagnostics().items():
            if k in ("QF Unordered", "QF target Undordered"):   # integer counts: exact
                assert v == float(g[f"s{s}/stat/{k}"]), (k, v, g[f"s{s}/stat/{k}"])
                continue
            errs[f"s{s}/stat/{k}"] = parity.stat_err(v, g, f"s{s}/stat/{k}")
    # every step under the noise-derived gate (max(1e-5, 3x the reference's
    # own fp32 distance from the float64 oracle, per key))
    noise = tog.ptrain_errors(meta, g, tog.make_ptrain_oracle(meta, torch.float64, g=g))
    bad = tog.gated(errs, noise)
    print(name, "worst", sorted(errs.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def test_ptrain_stats_keys_match_reference_order():
    meta, g = parity.load("ptrain_small")
    tr = ptrain_trainer_for(meta)
    tr.train_from_torch(batch_from(meta, g["s0/idx"]))
    keys = [k[len("s0/stat/"):] for k in g if k.startswith("s0/stat/")]
    assert list(tr.get_diagnostics().keys()) == keys


@pytest.mark.parametrize("B", [1024, 4096])
def test_ptrain_large_batch_matches_oracle(B):
    """Humanoid dims, K=10 (reproduce_p-oac_humanoid_counts.sh) at the
    large-batch kernel configuration: one step against the fp32 CPU oracle on
    the same inputs (tolerance 1e-5 on every gradient tensor)."""
    from oracle import sac_oracle as so
    Do, Da, H, K = 376, 17, [256, 256], 10
    meta = dict(obs_dim=Do, act_dim=Da, hidden=H, seed=5, K=K, q_min=0.0, q_max=500.0,
                pi_init_w=1e-3, q_init_w=3e-3, discount=0.99, delta=0.95, lr=3e-4, tau=5e-3,
                counts=True, n_replay=20000)
    params = ptrain_params(Do, Da, H, meta["seed"], K, 0.0, 500.0)
    tr = ptrain_trainer_for(meta, params=params)
    rs = np.random.RandomState(B)
    b = batch_from(meta, rs.randint(0, meta["n_replay"], B))
    b["counts"] = (rs.randint(0, 3, (B, 1)) * (rs.uniform(0, 1, (B, 1)) < 0.5)).astype(np.float64)
    tr.train_from_torch(b)
    torch.cuda.synchronize()
    orc = so.ParticleUBOracle(params, Do, Da, K, tr.delta_index, q_min=0.0, q_max=500.0,
                              policy_lr=3e-4, qf_lr=3e-4, tau=5e-3)
    out = orc.step(b)
    worst = {}
    for grp, mod, order in (("policy", tr.policy, PARAM_ORDER_POLICY[:6]),
                            ("target_policy", tr.target_policy, PARAM_ORDER_POLICY[:6]),
                            ("qf", tr.qfs[0], PARAM_ORDER_Q)):
        gv = module_tensors(tr, mod, tr.grads)
        for pn in order:
            worst[f"{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(),
                                                  out["grads"][grp][pn].numpy())
    bad = {k: v for k, v in worst.items() if v > 1e-5}
    print(B, sorted(worst.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, bad
