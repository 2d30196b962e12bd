"""GPU parity of the g-oac GaussianTrainer (share_layers critic [Q | log std],
deterministic policy, target_policy) against the reference's own outputs
(tests/golden/goac_*.npz, make_golden.py gen_goac) and, at the large-batch
kernel configuration, against the CPU oracle."""
import numpy as np
import pytest
import torch

import parity
import test_oracle_golden as tog
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q, goac_params
from gpu_helpers import Space, StateDictModule, batch_from, module_tensors

pytestmark = pytest.mark.gpu

FIXTURES = ["goac_small", "goac_counts", "goac_soft", "goac_humanoid", "goac_nobias",
            "goac_tpn"]


def goac_producers(params):
    """Producers in the reference constructor's call order: SACTrainer's
    policy and four critics, the shared-layer critic and its target, then
    target_policy (gaussian_trainer.py:51-63, 91-99, 146)."""
    # a third policy_producer() call builds use_target_policy's network (its
    # weights are then overwritten: a copy of the policy, then the fixture's)
    pols = iter([params["policy"], params["target_policy"], params["policy"]])
    qs = iter([params["qf1"]] * 4 + [params["qf1"], params["target_qf1"]])
    return (lambda **k: StateDictModule(next(pols)),
            lambda **k: StateDictModule(next(qs)))


def goac_trainer_for(meta, params=None, **kw):
    from oac_amd import GaussianTrainer
    if params is None:
        params = goac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                             meta["q_min"], meta["q_max"], pi_init_w=meta["pi_init_w"],
                             q_init_w=meta["q_init_w"])
    pp, qp = goac_producers(params)
    soft = meta.get("soft")
    return GaussianTrainer(pp, qp, n_estimators=2, action_space=Space(meta["act_dim"]),
                           discount=meta["discount"], reward_scale=1.0, delta=meta["delta"],
                           policy_lr=meta["lr"], qf_lr=meta["lr"], soft_target_tau=meta["tau"],
                           target_update_period=1, q_min=meta["q_min"], q_max=meta["q_max"],
                           share_layers=True, counts=bool(meta.get("counts")),
                           std_soft_update=soft is not None,
                           std_soft_update_prob=0.0 if soft is None else soft,
                           train_bias=meta.get("train_bias", True),
                           use_target_policy=bool(meta.get("use_target_policy")), **kw)


@pytest.mark.parametrize("name", FIXTURES)
def test_goac_step_matches_reference_golden(name):
    meta, g = parity.load(name)
    tr = goac_trainer_for(meta)
    if meta.get("use_target_policy"):   # the fixture's DDPG target network weights
        tr.target_policy_network.load_state_dict(
            {k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("tpn/")})
    assert abs(tr.standard_bound - meta["standard_bound"]) < 1e-12
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
                                ("qf", tr.q, PARAM_ORDER_Q)):
            gv = module_tensors(tr, mod, tr.grads)
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, gv[pn].cpu().numpy())
        for grp, mod in (("policy", tr.policy), ("target_policy", tr.target_policy),
                         ("qf", tr.q), ("tf", tr.q_target)):
            for pn, t in mod.state_dict().items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.cpu().numpy(), meta["lr"])
        for k, v in tr.get_diagnostics().items():
            errs[f"s{s}/stat/{k}"] = parity.stat_err(v, g, f"s{s}/stat/{k}")
    # every step under the noise-derived gate (max(1e-5, 3x the reference's
    # own fp32 distance from the float64 oracle, per key))
    noise = tog.goac_errors(meta, g, tog.make_goac_oracle(meta, torch.float64, g=g))
    bad = tog.gated(errs, noise)
    print(name, "worst", sorted(errs.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def test_goac_stats_keys_match_reference_order():
    meta, g = parity.load("goac_small")
    tr = goac_trainer_for(meta)
    tr.train_from_torch(batch_from(meta, g["s0/idx"]))
    keys = [k[len("s0/stat/"):] for k in g if k.startswith("s0/stat/")]
    assert list(tr.get_diagnostics().keys()) == keys


def test_goac_log_std_heads_untouched_and_snapshot_keys():
    """The deterministic policies' log-std heads get no gradient, so Adam
    leaves them bit-identical and keeps no state for them (torch skips
    parameters whose grad is None); snapshot keys are the reference's."""
    meta, g = parity.load("goac_small")
    tr = goac_trainer_for(meta)
    before = {k: v.clone() for k, v in tr.policy.state_dict().items()}
    tr.train_from_torch(batch_from(meta, g["s0/idx"]))
    torch.cuda.synchronize()
    after = tr.policy.state_dict()
    for k in ("last_fc_log_std.weight", "last_fc_log_std.bias"):
        assert torch.equal(before[k], after[k]), k
    ss = tr.get_snapshot()
    assert set(ss) == {"policy_state_dict", "policy_optim_state_dict", "log_alpha",
                       "alpha_optim_state_dict", "eval_statistics", "_n_train_steps_total",
                       "_need_to_update_eval_statistics", "qfs_state_dicts",
                       "qfs_optims_state_dicts", "target_qfs_state_dicts",
                       "target_policy_state_dict", "target_policy_opt_state_dict"}
    assert sorted(ss["policy_optim_state_dict"]["state"]) == [0, 1, 2, 3, 4, 5]


@pytest.mark.parametrize("B", [1024, 4096])
def test_goac_large_batch_matches_oracle(B):
    """Humanoid dims at the large-batch kernel configuration (register-direct
    forward GEMMs, split-K weight gradients): one step against the fp32 CPU
    oracle on the same inputs (tolerance 1e-5 on every gradient tensor)."""
    from oracle import sac_oracle as so
    Do, Da, H = 376, 17, [256, 256]
    meta = dict(obs_dim=Do, act_dim=Da, hidden=H, seed=5, q_min=0.0, q_max=500.0,
                pi_init_w=1e-3, q_init_w=3e-3, discount=0.99, delta=0.95, lr=3e-4, tau=5e-3,
                counts=True, n_replay=20000)
    params = goac_params(Do, Da, H, meta["seed"], 0.0, 500.0)
    tr = goac_trainer_for(meta, params=params)
    rs = np.random.RandomState(B)
    b = batch_from(meta, rs.randint(0, meta["n_replay"], B))
    b["counts"] = (rs.randint(0, 3, (B, 1)) * (rs.uniform(0, 1, (B, 1)) < 0.5)).astype(np.float64)
    tr.train_from_torch(b)
    torch.cuda.synchronize()
    orc = so.GaussianOACOracle(params, Do, Da, delta=0.95, q_min=0.0, q_max=500.0,
                               policy_lr=3e-4, qf_lr=3e-4, tau=5e-3)
    out = orc.step(b)
    worst = {}
    for grp, mod, order in (("policy", tr.policy, PARAM_ORDER_POLICY[:6]),
                            ("target_policy", tr.target_policy, PARAM_ORDER_POLICY[:6]),
                            ("qf", tr.q, PARAM_ORDER_Q)):
        gv = module_tensors(tr, mod, tr.grads)
        for pn in order:
            worst[f"{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(),
                                                  out["grads"][grp][pn].numpy())
    bad = {k: v for k, v in worst.items() if v > 1e-5}
    print(B, sorted(worst.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, bad
