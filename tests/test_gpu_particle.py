"""GPU parity of the P-OAC particle trainer (share_layers K-head critic)
against the reference's own outputs (tests/golden/poac_*.npz)."""
import numpy as np
import pytest
import torch

import parity
import test_oracle_golden as tog
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q, sac_params
from gpu_helpers import Space, batch_from, module_tensors, producers

pytestmark = pytest.mark.gpu


def particle_trainer_for(meta, **kw):
    from oac_amd import ParticleTrainerOAC as ParticleTrainer
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"], q_out=K,
                        q_last_bias=np.linspace(meta["q_min"], meta["q_max"], K),
                        pi_init_w=meta["pi_init_w"])
    pp, qp = producers(params, q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                       "target_qf1"))
    return ParticleTrainer(pp, qp, n_estimators=K, action_space=Space(meta["act_dim"]),
                           discount=meta["discount"], reward_scale=1.0, delta=meta["delta"],
                           policy_lr=meta["lr"], qf_lr=meta["lr"], soft_target_tau=meta["tau"],
                           target_update_period=meta.get("target_update_period", 1),
                           use_automatic_entropy_tuning=True,
                           deterministic=False, q_min=meta["q_min"], q_max=meta["q_max"],
                           share_layers=True, train_bias=meta.get("train_bias", True), **kw)


@pytest.mark.parametrize("name", ["poac_small", "poac_ant", "poac_ant_b4096", "poac_counts",
                                  "poac_nobias", "poac_period2"])
def test_particle_step_matches_reference_golden(name):
    meta, g = parity.load(name)
    tr = particle_trainer_for(meta, counts=bool(meta.get("counts")))
    assert tr.delta_index == meta["delta_index"]
    errs = {}
    for s in range(meta["steps"]):
        tr.end_epoch(s)
        b = batch_from(meta, g[f"s{s}/idx"])
        if meta.get("counts"):
            b["counts"] = g[f"s{s}/counts"][:, None]
        tr.train_from_torch(b, eps1=g[f"s{s}/eps1"], eps2=g[f"s{s}/eps2"])
        torch.cuda.synchronize()
        for grp, mod, order in (("policy", tr.policy, PARAM_ORDER_POLICY),
                                ("qf", tr.qfs[0], PARAM_ORDER_Q)):
            gv = module_tensors(tr, mod, tr.grads)
            for pn in order:
                key = f"s{s}/grad/{grp}/{pn}"
                errs[key] = parity.compare(g, key, gv[pn].cpu().numpy())
        a = tr.alpha_state.cpu().numpy()
        errs[f"s{s}/grad/log_alpha"] = parity.rel_err(a[5:6], g[f"s{s}/grad/log_alpha"])
        errs[f"s{s}/post/log_alpha"] = parity.rel_err(a[0:1], g[f"s{s}/post/log_alpha"])
        for grp, mod in (("policy", tr.policy), ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
            for pn, t in mod.state_dict().items():
                key = f"s{s}/post/{grp}/{pn}"
                gk = f"s{s}/grad/{grp}/{pn}" if s == 0 and grp != "tf" else None
                errs[key], _ = parity.compare_post(g, key, gk, t.cpu().numpy(), meta["lr"])
        st = tr.get_diagnostics()
        for k in list(st.keys()):
            gk = f"s{s}/stat/{k}"
            if k in tog.COUNT_STATS:   # integer counts: exact
                assert st[k] == float(g[gk]), (k, st[k], g[gk])
            elif gk in g:
                errs[gk] = parity.stat_err(st[k], g, gk)
    # every step under the noise-derived gate: max(1e-5, 3x the reference's
    # own fp32 distance from the float64 oracle, per key)
    noise = tog.poac_noise(meta, g)
    bad = tog.gated(errs, noise)
    print(name, "worst", sorted(errs.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]


def test_particle_step_with_a_nan_head_sorts_it_last():
    """A diverged head (NaN Q values in every row): the targets kernel's rank
    sort puts NaN after every number, as torch.sort does
    (particle_trainer_oac.py:192, 202), so each slot is taken once and the
    dq / LDS scatters stay inside the K heads.  The finite slots' losses equal
    the oracle's (torch.sort on the same NaN head); the NaN slot's loss is NaN."""
    meta, g = parity.load("poac_small")
    K = meta["K"]
    tr = particle_trainer_for(meta)
    with torch.no_grad():
        tr.qfs[0].state_dict()["last_fc.weight"][K // 2].fill_(float("nan"))
    orc = tog.make_poac_oracle(meta)
    orc.Q["last_fc.weight"][K // 2] = float("nan")
    b = batch_from(meta, g["s0/idx"])
    tr.end_epoch(0)
    tr.train_from_torch(b, eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    torch.cuda.synchronize()
    out = orc.step(b, g["s0/eps1"], g["s0/eps2"])
    st = tr.get_diagnostics()
    for i in range(K - 1):
        ref = float(out["qf_losses"][i])
        assert np.isfinite(ref) and parity.rel_err(st[f"QF{i} Loss"], ref) < 1e-5, (i, st[f"QF{i} Loss"], ref)
    assert np.isnan(st[f"QF{K - 1} Loss"]) and np.isnan(float(out["qf_losses"][K - 1]))
    # the trainer keeps stepping (no fault, no stale LDS slot)
    tr.train_from_torch(b, eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    torch.cuda.synchronize()


def test_particle_stats_keys_match_reference_order():
    meta, g = parity.load("poac_small")
    tr = particle_trainer_for(meta)
    tr.train_from_torch(batch_from(meta, g["s0/idx"]), eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    keys = [k[len("s0/stat/"):] for k in g if k.startswith("s0/stat/")]
    assert list(tr.get_diagnostics().keys()) == keys


@pytest.mark.parametrize("B", [1024, 4096])
def test_particle_large_batch_matches_oracle(B):
    """BASELINE configs[4] (particle_trainer_oac K=10, Ant-v2 dims, batch
    4096) on the large-batch kernels (the LDS-DMA pipelined forward and
    backward GEMMs, gemm_fwd.hip / gemm_bwdp.hip, incl. the post-step critic
    layer 0 on a~ as a rank-R continuation; narrow products on the small-tile
    kernel): one step against the fp32 CPU oracle on the same inputs and
    eps: 1e-5 on every gradient tensor, on the post-step parameters (Adam's
    sign band aside, parity.compare_post), the Adam moments, the target
    critic after Polyak, log-alpha and its gradient, and the K head losses."""
    from oracle import sac_oracle as so
    from gpu_helpers import batch_from
    meta = dict(obs_dim=111, act_dim=8, hidden=[256, 256], K=10, seed=11, q_min=0.0,
                q_max=500.0, pi_init_w=1e-3, lr=3e-4, tau=5e-3, discount=0.99, delta=0.95,
                n_replay=20000)
    K, lr = meta["K"], meta["lr"]
    params = sac_params(111, 8, [256, 256], meta["seed"], q_out=K,
                        q_last_bias=np.linspace(0.0, 500.0, K), pi_init_w=1e-3)
    tr = particle_trainer_for(meta)
    rs = np.random.RandomState(B)
    b = batch_from(meta, rs.randint(0, meta["n_replay"], B))
    e1 = rs.standard_normal((B, 8)).astype(np.float32)
    e2 = rs.standard_normal((B, 8)).astype(np.float32)
    tr.end_epoch(0)
    tr.train_from_torch(b, eps1=e1, eps2=e2)
    torch.cuda.synchronize()
    orc = so.ParticleOACOracle(params, 111, 8, K, policy_lr=lr, qf_lr=lr)
    out = orc.step(b, e1, e2)

    def post_err(got, ref, grad, band=1e-3):
        got, ref, grad = (np.asarray(x, np.float64).reshape(-1) for x in (got, ref, grad))
        rms = np.sqrt(np.mean(grad * grad))
        ok = np.abs(grad) > band * rms
        d = got - ref
        assert np.all(np.abs(d[~ok]) <= 2.5 * lr + 1e-6)   # Adam's first step ~ lr sign(g)
        return np.linalg.norm(d[ok]) / np.linalg.norm(ref)

    worst = {}
    for grp, mod, order, opt in (("policy", tr.policy, PARAM_ORDER_POLICY, orc.opt_p),
                                 ("qf", tr.qfs[0], PARAM_ORDER_Q, orc.opt_q)):
        gv = module_tensors(tr, mod, tr.grads)
        mv = module_tensors(tr, mod, tr.adam_m)
        vv = module_tensors(tr, mod, tr.adam_v)
        pv = dict(mod.state_dict())
        for pn in order:
            gref = out["grads"][grp][pn].numpy()
            worst[f"grad/{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(), gref)
            worst[f"m/{grp}/{pn}"] = parity.rel_err(mv[pn].cpu().numpy(), opt.m[pn].numpy())
            worst[f"v/{grp}/{pn}"] = parity.rel_err(vv[pn].cpu().numpy(), opt.v[pn].numpy())
            ref = (orc.P if grp == "policy" else orc.Q)[pn].numpy()
            worst[f"post/{grp}/{pn}"] = post_err(pv[pn].cpu().numpy(), ref, gref)
    for pn, t in tr.tfs[0].state_dict().items():
        worst[f"post/tf/{pn}"] = parity.rel_err(t.cpu().numpy(), orc.T[pn].numpy())
    a = tr.alpha_state.cpu().numpy()
    worst["grad/log_alpha"] = parity.rel_err(a[5:6], out["grads"]["log_alpha"].numpy())
    worst["post/log_alpha"] = parity.rel_err(a[0:1], orc.log_alpha.numpy())
    st = tr.get_diagnostics()
    for i in range(K):
        worst[f"QF{i} Loss"] = parity.rel_err(st[f"QF{i} Loss"], float(out["qf_losses"][i]))
    worst["Policy Loss"] = parity.rel_err(st["Policy Loss"], float(out["policy_loss"]))
    bad = {k: v for k, v in worst.items() if v > 1e-5}
    print(B, sorted(worst.items(), key=lambda kv: -kv[1])[:3])
    assert not bad, bad
