"""Teacher-forced per-step parity at the BASELINE dims.

The trajectory tests (test_gpu_parity.py, test_gpu_particle.py) run the GPU
trainer through a reference fixture's steps and gate every key at
max(1e-5, 3 x the reference's own fp32 noise): past step 0 the fp32
trajectories of two correct implementations drift apart (Adam's first step is
lr * sign(g), ReLU masks flip), so that gate widens to ~1e-2 for some keys at
Humanoid dims.  Here every step is checked at the north_star's 1e-5 instead:
before step s the GPU trainer's OWN pre-step state -- parameters, target
critics, Adam m / v and step count, log-alpha and its Adam state -- is loaded
into the fp32 CPU oracle, both take step s on the fixture's batch and eps
(reference-drawn), and gradients, post-step parameters, Adam moments, Polyak
targets, log-alpha (gradient and value) and the losses are compared.

Allowances, each reported by the test: elements of a post-step parameter
whose gradient is within fp32 rounding of 0 (Adam moves them by ~lr * sign,
bounded by 2.5 lr); at most two rows of a critic hidden-layer gradient whose
ReLU pre-activation sits within fp32 rounding of 0 for some sample
(parity.relu_boundary_units), as in test_gpu_dp.py; for a SAC critic's first
layer, the layer-1 mask flips, which reach every fc0 row (_flip_adjusted: the
(sample, unit) entries where the GPU's own saved layer-1 activations -- the
masks its backward used, workspace views h2q1 / h2q2 -- disagree in sign with
the oracle's are listed, each is asserted to sit within 3e-5 rms of 0, the
oracle's fc0 reference is corrected by exactly those entries, and the result
is gated at 1e-5); and the same rule for BOTH hidden layers of the policy
(_policy_flip_adjusted, workspace views h1p / h2p), with no policy row left
out (sac_humanoid_b4096 step 2 has a policy layer-0 unit at 6.7e-7 rms of 0
that takes the other sign under the chunked slab order of the round-5 Adam
launch, tools/diag_teacher_flip.py).

The drop-in tests (test_*_dropin_teacher_forced) do the same on the call path
the bench times -- ReplayBuffer.random_batch + trainer.train, i.e. host
indices staged into the step's first launch, device Philox eps, the deferred
layer-0 Adam -- reading each step's eps back from the plan's workspace and
checking the in-step gather against the replay rows bit for bit.

Reference: trainer/trainer.py:126-280 (SAC), trainer/particle_trainer_oac.py:
169-363 (P-OAC), torch-1.4 Adam (trainer/trainer.py:75-91).
"""
import numpy as np
import pytest
import torch

import parity
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q
from gpu_helpers import batch_from, module_tensors, sac_trainer_for
from oracle import sac_oracle as so

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _np_sd(mod):
    return {k: v.detach().cpu().numpy().copy() for k, v in mod.state_dict().items()}


def _load_adam(opt, tr, mod):
    m = module_tensors(tr, mod, tr.adam_m)
    v = module_tensors(tr, mod, tr.adam_v)
    for k in opt.m:
        opt.m[k].copy_(m[k].detach().cpu())
        opt.v[k].copy_(v[k].detach().cpu())
    opt.t = tr._n_train_steps_total


def _load_alpha(orc, tr):
    a = tr.alpha_state.detach().cpu()
    orc.log_alpha.copy_(a[0:1])
    orc.opt_a.m["log_alpha"].copy_(a[1:2])
    orc.opt_a.v["log_alpha"].copy_(a[2:3])
    orc.opt_a.t = tr._n_train_steps_total
    orc.n_steps = tr._n_train_steps_total


def sac_oracle_from_gpu(tr, meta):
    """The fp32 oracle holding the GPU SAC trainer's current state."""
    params = {g: _np_sd(getattr(tr, g))
              for g in ("policy", "qf1", "qf2", "target_qf1", "target_qf2")}
    orc = so.SACOracle(params, meta["obs_dim"], meta["act_dim"], discount=meta["discount"],
                       reward_scale=meta["reward_scale"], policy_lr=meta["lr"],
                       qf_lr=meta["lr"], tau=meta["tau"], auto_alpha=meta["auto_alpha"],
                       target_update_period=meta.get("target_update_period", 1))
    for opt, mod in ((orc.opt_p, tr.policy), (orc.opt_q1, tr.qf1), (orc.opt_q2, tr.qf2)):
        _load_adam(opt, tr, mod)
    _load_alpha(orc, tr)
    return orc


def poac_oracle_from_gpu(tr, meta):
    params = {"policy": _np_sd(tr.policy), "qf1": _np_sd(tr.qfs[0]),
              "target_qf1": _np_sd(tr.tfs[0])}
    orc = so.ParticleOACOracle(params, meta["obs_dim"], meta["act_dim"], meta["K"],
                               discount=meta["discount"], policy_lr=meta["lr"],
                               qf_lr=meta["lr"], tau=meta["tau"],
                               target_update_period=meta.get("target_update_period", 1),
                               train_bias=meta.get("train_bias", True))
    _load_adam(orc.opt_p, tr, tr.policy)
    _load_adam(orc.opt_q, tr, tr.qfs[0])
    _load_alpha(orc, tr)
    return orc


def _post_err(got, ref, grad, lr, band=1e-3):
    """Norm-relative error of a post-step parameter outside Adam's sign band;
    band elements bounded by 2.5 lr.  Returns (err, band elements)."""
    got, ref, grad = (np.asarray(x, np.float64).reshape(-1) for x in (got, ref, grad))
    rms = np.sqrt(np.mean(grad * grad)) if grad.size else 0.0
    ok = np.abs(grad) > band * rms
    d = got - ref
    assert np.all(np.abs(d[~ok]) <= 2.5 * lr + 1e-6)
    n = np.linalg.norm(ref)
    return (np.linalg.norm(d[ok]) / n if n else np.linalg.norm(d[ok])), int((~ok).sum())


def _boundary_rows(x0, q):
    """ReLU-boundary hidden units of a critic on input rows x0 (both layers)."""
    u0, pre0 = parity.relu_boundary_units(x0, q["fc0.weight"], q["fc0.bias"])
    u1, _ = parity.relu_boundary_units(np.maximum(pre0, 0), q["fc1.weight"], q["fc1.bias"])
    return {"fc0.weight": u0, "fc0.bias": u0, "fc1.weight": u1, "fc1.bias": u1}


def _flip_adjusted(gref, cache, dq, q, opt, lr, gpu_h2, tol=3e-5):
    """fc0 references under the GPU's own layer-1 ReLU masks.

    A layer-1 pre-activation within fp32 rounding of 0 for sample s, unit u
    may take the other sign on the GPU; the backward then passes (or stops)
    that sample's dL/dpre1[s, u] = dq[s] . W_last[:, u], which reaches EVERY
    fc0 row through W1[u, :] (a rank-one change dd0 x[s]^T).  The flipped
    entries are read off the GPU's saved layer-1 activations (``gpu_h2``, the
    masks its backward used) against the oracle's; each must sit within
    ``tol`` rms of 0 (else the GPU computed a different layer, not a rounding
    flip), and the fc0 reference is corrected by exactly those entries -- m,
    v and the post-step fc0 follow through torch-1.4 Adam in float64.  The fc1
    rows u are allowed separately (_boundary_rows).  Returns ({pn: (g, m, v,
    P)}, flipped entries)."""
    x = cache["hs"][0].double().numpy()
    h1 = cache["hs"][1].double().numpy()
    h2 = cache["hs"][2].numpy()
    W1 = np.asarray(q["fc1.weight"], np.float64)
    pre1 = h1 @ W1.T + np.asarray(q["fc1.bias"], np.float64)
    rms = np.sqrt(np.mean(pre1 * pre1))
    flips = np.argwhere((h2 > 0) != (np.asarray(gpu_h2) > 0))
    far = [(int(s_), int(u), float(abs(pre1[s_, u]) / rms)) for s_, u in flips
           if abs(pre1[s_, u]) >= tol * rms]
    assert not far, ("layer-1 masks differ away from 0 (sample, unit, |pre1| / rms)", far[:8])
    dqn = dq.double().numpy().reshape(dq.shape[0], -1)
    wl = np.asarray(q["last_fc.weight"], np.float64)
    sel = []
    for s_, u in flips:
        val = float(dqn[s_] @ wl[:, u])
        sign = -1.0 if h2[s_, u] > 0 else 1.0
        dd0 = sign * val * W1[u] * (h1[s_] > 0)
        sel.append(((int(s_), int(u)), np.outer(dd0, x[s_]), dd0))
    out = {}
    t = opt.t
    bc1, bc2 = 1 - opt.b1 ** t, 1 - opt.b2 ** t
    for pn, k in (("fc0.weight", 1), ("fc0.bias", 2)):
        g = gref[pn].double().numpy()
        dg = sum(d[k] for d in sel) if sel else np.zeros_like(g)
        m = opt.m[pn].double().numpy() + (1 - opt.b1) * dg
        v = opt.v[pn].double().numpy() + (1 - opt.b2) * (2 * g * dg + dg * dg)
        P = np.asarray(q[pn], np.float64) - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + opt.eps)
        out[pn] = (g + dg, m, v, P)
    return out, [d[0] for d in sel]


def _policy_flip_adjusted(gref, pf, up, p, opt, lr, gpu_h1, gpu_h2, tol=3e-5):
    """Policy trunk references under the GPU's own ReLU masks.

    The critics' rule (_flip_adjusted) for both hidden layers of the policy:
    the (layer, sample, unit) entries where the GPU's saved activations on
    obs (workspace views h1p / h2p: the masks its policy backward used)
    disagree in sign with the oracle's are listed, each must sit within
    ``tol`` rms of 0, and the fc0 / fc1 references are recomputed in float64
    under the GPU's masks (the heads' upstream gradients ``up`` = (dL/da,
    dL/dlogp) and the pre-step weights ``p`` as the oracle had them); the
    difference is added to the oracle's fp32 gradients and m, v and the
    post-step parameters follow through torch-1.4 Adam.  A flipped entry's
    activation is within rounding of 0 either way, so the heads' gradients
    are unchanged.  Returns ({pn: (g, m, v, P)}, flipped entries)."""
    f64 = lambda t: (t.double().numpy() if torch.is_tensor(t) else np.asarray(t, np.float64))
    x, h1, h2 = (f64(pf["hs"][i]) for i in range(3))
    W0, b0, W1, b1 = (f64(p[k]) for k in ("fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias"))
    pre = (x @ W0.T + b0, h1 @ W1.T + b1)
    mo = (f64(pf["hs"][1]) > 0, f64(pf["hs"][2]) > 0)
    mg = (np.asarray(gpu_h1) > 0, np.asarray(gpu_h2) > 0)
    flips = []
    for l in range(2):
        rms = np.sqrt(np.mean(pre[l] * pre[l]))
        fl = np.argwhere(mo[l] != mg[l])
        far = [(l, int(s_), int(u), float(abs(pre[l][s_, u]) / rms)) for s_, u in fl
               if abs(pre[l][s_, u]) >= tol * rms]
        assert not far, ("policy masks differ away from 0 (layer, sample, unit, |pre| / rms)",
                         far[:8])
        flips += [(l, int(s_), int(u)) for s_, u in fl]
    if not flips:
        return {}, []
    dmean, dls = so.policy_head_grads(pf, *up)
    dh2 = f64(dmean) @ f64(p["last_fc.weight"]) + f64(dls) @ f64(p["last_fc_log_std.weight"])

    def trunk(m1, m2):
        d1 = dh2 * m2
        d0 = (d1 @ W1) * m1
        return {"fc0.weight": d0.T @ x, "fc0.bias": d0.sum(0),
                "fc1.weight": d1.T @ h1, "fc1.bias": d1.sum(0)}

    go, gg = trunk(*mo), trunk(*mg)
    out = {}
    t = opt.t
    bc1, bc2 = 1 - opt.b1 ** t, 1 - opt.b2 ** t
    for pn in go:
        g = gref[pn].double().numpy()
        dg = gg[pn] - go[pn]
        m = opt.m[pn].double().numpy() + (1 - opt.b1) * dg
        v = opt.v[pn].double().numpy() + (1 - opt.b2) * (2 * g * dg + dg * dg)
        P = np.asarray(p[pn], np.float64) - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + opt.eps)
        out[pn] = (g + dg, m, v, P)
    return out, flips


def _compare_group(errs, left_out, tr, mod, grp, order, opt, P, grads, lr, allowed, flip=None,
                   pflip=None):
    """Gradient, Adam m / v and post-step errors of one module's parameters
    (ReLU-boundary rows as allowed; with ``flip`` = (forward cache, dq,
    pre-step params, the GPU's layer-1 activations) a critic's fc0
    references take the GPU's layer-1 mask flips, _flip_adjusted; with
    ``pflip`` = (policy forward cache, upstream gradients, pre-step params,
    the GPU's h1 / h2) the policy's fc0 / fc1 take its mask flips,
    _policy_flip_adjusted)."""
    gv = module_tensors(tr, mod, tr.grads)
    mv = module_tensors(tr, mod, tr.adam_m)
    vv = module_tensors(tr, mod, tr.adam_v)
    sd = dict(mod.state_dict())
    refs = {pn: (grads[pn].numpy(), opt.m[pn].numpy(), opt.v[pn].numpy(), P[pn].numpy())
            for pn in order}
    if flip is not None and "fc1.weight" in order:
        cache, dq, q, gpu_h2 = flip
        adj, flips = _flip_adjusted(grads, cache, dq, q, opt, lr, gpu_h2)
        if flips:
            refs.update(adj)
            left_out[f"{grp}/layer-1 mask flips (sample, unit)"] = flips
    if pflip is not None:
        pfc, up, p, g1, g2 = pflip
        adj, flips = _policy_flip_adjusted(grads, pfc, up, p, opt, lr, g1, g2)
        if flips:
            refs.update(adj)
            left_out[f"{grp}/mask flips (layer, sample, unit)"] = flips
    for pn in order:
        gref, mref, vref, pref = refs[pn]
        e, bad = parity.rel_err_rows(gv[pn].cpu().numpy(), gref, allowed.get(pn, []))
        errs[f"grad/{grp}/{pn}"] = e
        if bad:
            left_out[f"{grp}/{pn}"] = bad
        keep = np.ones(gref.shape[0], bool)
        keep[bad] = False
        errs[f"m/{grp}/{pn}"] = parity.rel_err(mv[pn].cpu().numpy()[keep], mref[keep])
        errs[f"v/{grp}/{pn}"] = parity.rel_err(vv[pn].cpu().numpy()[keep], vref[keep])
        errs[f"post/{grp}/{pn}"], _ = _post_err(sd[pn].cpu().numpy()[keep], pref[keep],
                                                gref[keep], lr)


def _check(errs, left_out, name, s):
    bad = {k: v for k, v in errs.items() if v > TOL}
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
    print(f"{name} step {s}: worst {worst}; ReLU-boundary rows left out {left_out}")
    assert not bad, (name, s, sorted(bad.items(), key=lambda kv: -kv[1])[:10])


def _views(tr, *names):
    return [tr._last_plan.views[n].cpu().numpy() for n in names]


def _sac_compare(tr, orc, out, pre, batch, meta, name, s):
    """Every tensor of one SAC step against the oracle's step on the GPU's
    pre-step state (gate TOL; allowances in the module docstring)."""
    lr = meta["lr"]
    h2g = dict(zip(("qf1", "qf2"), _views(tr, "h2q1", "h2q2")))
    h1p, h2p = _views(tr, "h1p", "h2p")
    x0 = np.concatenate([batch["observations"], batch["actions"]], 1)
    allowed = {grp: _boundary_rows(x0, pre[grp]) for grp in ("qf1", "qf2")}
    B = x0.shape[0]
    dqs = {grp: 2.0 * (orc.S[c]["q"] - orc.S["y"]) / B for grp, c in (("qf1", "c1"), ("qf2", "c2"))}
    errs, left_out = {}, {}
    for grp, mod, order, opt, P in (("policy", tr.policy, PARAM_ORDER_POLICY, orc.opt_p, orc.P),
                                    ("qf1", tr.qf1, PARAM_ORDER_Q, orc.opt_q1, orc.Q1),
                                    ("qf2", tr.qf2, PARAM_ORDER_Q, orc.opt_q2, orc.Q2)):
        _compare_group(errs, left_out, tr, mod, grp, order, opt, P, out["grads"][grp], lr,
                       allowed.get(grp, {}),
                       (orc.S["c" + grp[-1]], dqs[grp], pre[grp], h2g[grp])
                       if grp in dqs else None,
                       (out["pf"], out["pol_up"], pre["policy"], h1p, h2p)
                       if grp == "policy" else None)
    for grp, mod, T in (("target_qf1", tr.target_qf1, orc.T1),
                        ("target_qf2", tr.target_qf2, orc.T2)):
        for pn, t in mod.state_dict().items():
            errs[f"post/{grp}/{pn}"] = parity.rel_err(t.cpu().numpy(), T[pn].numpy())
    if meta["auto_alpha"]:
        a = tr.alpha_state.cpu().numpy()
        errs["grad/log_alpha"] = parity.rel_err(a[5:6], out["grads"]["log_alpha"].numpy())
        errs["post/log_alpha"] = parity.rel_err(a[0:1], orc.log_alpha.numpy())
        errs["adam/log_alpha"] = parity.rel_err(a[1:3], np.concatenate(
            [orc.opt_a.m["log_alpha"].numpy(), orc.opt_a.v["log_alpha"].numpy()]))
    st = tr.get_diagnostics()
    for k in ("QF1 Loss", "QF2 Loss", "Q Loss", "Policy Loss", "Alpha", "Alpha Loss",
              "Log Pis Mean", "Q Targets Mean", "Q1 Predictions Mean"):
        if k in out["stats"]:
            errs[f"stat/{k}"] = parity.rel_err(st[k], out["stats"][k])
    _check(errs, left_out, name, s)


# every SAC fixture: each config flag (no alpha tuning, target period 2, the
# small / stress / RiverSwim dims) through the step's fused paths at 1e-5
@pytest.mark.parametrize("name", ["sac_humanoid", "sac_humanoid_b4096", "sac_small", "sac_stress",
                                  "sac_noalpha", "sac_riverswim", "sac_period2"])
def test_sac_teacher_forced_every_step(name):
    meta, g = parity.load(name)
    tr = sac_trainer_for(meta)
    for s in range(meta["steps"]):
        orc = sac_oracle_from_gpu(tr, meta)
        pre = {grp: _np_sd(getattr(tr, grp)) for grp in ("qf1", "qf2", "policy")}
        batch = batch_from(meta, g[f"s{s}/idx"])
        e1, e2 = g[f"s{s}/eps1"], g[f"s{s}/eps2"]
        tr.end_epoch(s)
        tr.train_from_torch(batch, eps1=e1, eps2=e2)
        torch.cuda.synchronize()
        out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
        _sac_compare(tr, orc, out, pre, batch, meta, name, s)


# ------------------------------------------------- the timed call path itself
def _replay_for(meta):
    """The fixture's replay (fixtures_lib.synthetic_transitions, seed 0) in an
    oac_amd.ReplayBuffer on the GPU."""
    from oac_amd import ReplayBuffer
    from fixtures_lib import synthetic_transitions
    from gpu_helpers import Space
    n = meta["n_replay"]
    rb = ReplayBuffer(n, Space(meta["obs_dim"]), Space(meta["act_dim"]), device="cuda:0")
    d = synthetic_transitions(n, meta["obs_dim"], meta["act_dim"], seed=0)
    rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                       rewards=d["rewards"], next_observations=d["next_observations"],
                       terminals=d["terminals"])])
    return rb


def _dropin_step(tr, rb, meta):
    """One rl_algorithm.py:160-167 call (random_batch, then train) on the
    drop-in path; returns the step's indices, host batch and the eps the
    step drew (read back from the plan's workspace).  The batch the step
    gathered must equal the replay rows at those indices bit for bit."""
    B = meta["B"]
    batch = rb.random_batch(B)
    idx = np.array(batch.host_indices, copy=True)
    batch["buffer"] = rb                      # rl_algorithm.py:166
    n0 = tr._n_train_steps_total
    tr.train(batch)
    torch.cuda.synchronize()
    assert tr._n_train_steps_total == n0 + 1
    plan = tr._last_plan
    assert plan is tr._dropin[(B, rb._storage.data_ptr())], "not the drop-in plan"
    e1, e2 = (plan.views[k].cpu().numpy().copy() for k in ("eps1", "eps2"))
    row = rb._storage.shape[1]
    got = plan.views["batch"][:, :row].cpu().numpy()
    assert np.array_equal(got, rb._storage[torch.as_tensor(idx, device=rb._storage.device)]
                          .cpu().numpy()), "in-step gather differs from the replay rows"
    return idx, batch_from(meta, idx), e1, e2


@pytest.mark.parametrize("name", ["sac_humanoid", "sac_humanoid_b4096"])
def test_sac_dropin_teacher_forced(name):
    """The bench's timed call (rb.random_batch(B) + tr.train(batch):
    oac_sac_step_host_idx -- indices in the first launch's arguments or the
    host slot, device Philox eps, the deferred layer-0 Adam) at the
    fixture's dims, every step at 1e-5 against the oracle on the GPU's own
    pre-step state.  Reference: rl_algorithm.py:160-167, trainer.py:126-224."""
    meta, _ = parity.load(name)
    tr = sac_trainer_for(meta)
    rb = _replay_for(meta)
    np.random.seed(5)
    for s in range(3):
        orc = sac_oracle_from_gpu(tr, meta)
        pre = {grp: _np_sd(getattr(tr, grp)) for grp in ("qf1", "qf2", "policy")}
        tr.end_epoch(s)
        idx, batch, e1, e2 = _dropin_step(tr, rb, meta)
        assert np.all(np.isfinite(e1)) and np.std(e1) > 0.5, "eps not drawn by the step"
        out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
        _sac_compare(tr, orc, out, pre, batch, meta, name + "/dropin", s)
    from oac_amd._lib import TRACE, lib
    bits = lib().oac_sac_trace(tr._last_plan.handle, 1)
    if meta["B"] <= 256:   # the headline step's form: fused Adam, the head's dX in the dL/da launch
        assert bits & TRACE["fused"] and bits & TRACE["head_dh2"], bits


def _particle_compare(tr, orc, out, pre, pre_p, batch, meta, name, s):
    lr, K = meta["lr"], meta["K"]
    h1p, h2p = _views(tr, "h1p", "h2p")
    x0 = np.concatenate([batch["observations"], batch["actions"]], 1)
    allowed = {"qf": _boundary_rows(x0, pre)}
    errs, left_out = {}, {}
    for grp, mod, order, opt, P in (("policy", tr.policy, PARAM_ORDER_POLICY, orc.opt_p, orc.P),
                                    ("qf", tr.qfs[0], PARAM_ORDER_Q, orc.opt_q, orc.Q)):
        _compare_group(errs, left_out, tr, mod, grp, order, opt, P, out["grads"][grp], lr,
                       allowed.get(grp, {}), None,
                       (out["pf"], out["pol_up"], pre_p, h1p, h2p) if grp == "policy" else None)
    for pn, t in tr.tfs[0].state_dict().items():
        errs[f"post/tf/{pn}"] = parity.rel_err(t.cpu().numpy(), orc.T[pn].numpy())
    a = tr.alpha_state.cpu().numpy()
    errs["grad/log_alpha"] = parity.rel_err(a[5:6], out["grads"]["log_alpha"].numpy())
    errs["post/log_alpha"] = parity.rel_err(a[0:1], orc.log_alpha.numpy())
    st = tr.get_diagnostics()
    for i in range(K):
        errs[f"stat/QF{i} Loss"] = parity.rel_err(st[f"QF{i} Loss"], float(out["qf_losses"][i]))
    errs["stat/Policy Loss"] = parity.rel_err(st["Policy Loss"], float(out["policy_loss"]))
    _check(errs, left_out, name, s)


@pytest.mark.parametrize("name", ["poac_ant", "poac_ant_b4096", "poac_small", "poac_counts",
                                  "poac_nobias", "poac_period2"])
def test_particle_teacher_forced_every_step(name):
    from test_gpu_particle import particle_trainer_for
    meta, g = parity.load(name)
    tr = particle_trainer_for(meta)
    for s in range(meta["steps"]):
        orc = poac_oracle_from_gpu(tr, meta)
        pre, pre_p = _np_sd(tr.qfs[0]), _np_sd(tr.policy)
        batch = batch_from(meta, g[f"s{s}/idx"])
        e1, e2 = g[f"s{s}/eps1"], g[f"s{s}/eps2"]
        tr.end_epoch(s)
        tr.train_from_torch(batch, eps1=e1, eps2=e2)
        torch.cuda.synchronize()
        out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
        _particle_compare(tr, orc, out, pre, pre_p, batch, meta, name, s)


def test_particle_dropin_teacher_forced():
    """BASELINE configs[4] (K=10 shared-head critic, Ant-v2 dims, B=4096) on
    the bench's timed call (random_batch + train: host indices read by the
    step's first launch, device Philox eps), every step at 1e-5 against the
    oracle on the GPU's own pre-step state.  Reference:
    trainer/particle_trainer_oac.py:169-363, rl_algorithm.py:160-167."""
    from test_gpu_particle import particle_trainer_for
    meta, _ = parity.load("poac_ant_b4096")
    tr = particle_trainer_for(meta)
    rb = _replay_for(meta)
    np.random.seed(6)
    for s in range(2):
        orc = poac_oracle_from_gpu(tr, meta)
        pre, pre_p = _np_sd(tr.qfs[0]), _np_sd(tr.policy)
        tr.end_epoch(s)
        idx, batch, e1, e2 = _dropin_step(tr, rb, meta)
        assert np.all(np.isfinite(e1)) and np.std(e1) > 0.5, "eps not drawn by the step"
        out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
        _particle_compare(tr, orc, out, pre, pre_p, batch, meta, "poac_ant_b4096/dropin", s)


# ------------------------------------------------- mid-training-state goldens
def _optim_sd(mod, st, t):
    """torch-Adam state_dict of a module's parameters from mid_state moments."""
    state = {i: dict(step=t, exp_avg=torch.from_numpy(st[n][0].copy()),
                     exp_avg_sq=torch.from_numpy(st[n][1].copy()))
             for i, (n, _) in enumerate(mod.named_parameters())}
    return dict(state=state, param_groups=[dict(params=list(range(len(state))))])


def _alpha_sd(ms):
    am, av = ms["alpha_adam"]
    return dict(state={0: dict(step=ms["t"], exp_avg=torch.tensor([am]),
                               exp_avg_sq=torch.tensor([av]))},
                param_groups=[dict(params=[0])])


def _golden_errors(g, tr, groups, meta):
    """One-step errors against a mid-state golden: gradients (whole),
    post-step parameters, targets and Adam moments (sampled), log-alpha."""
    errs = {}
    for grp, mod, order in groups:
        gv = module_tensors(tr, mod, tr.grads)
        mv = module_tensors(tr, mod, tr.adam_m)
        vv = module_tensors(tr, mod, tr.adam_v)
        for pn in order:
            errs[f"grad/{grp}/{pn}"] = parity.compare(g, f"s0/grad/{grp}/{pn}",
                                                      gv[pn].cpu().numpy())
            for nm, t in (("exp_avg", mv[pn]), ("exp_avg_sq", vv[pn])):
                key = f"s0/adam/{grp}/{pn}/{nm}"
                errs[key] = parity.compare(g, key, t.cpu().numpy())
    a = tr.alpha_state.cpu().numpy()
    errs["grad/log_alpha"] = parity.rel_err(a[5:6], g["s0/grad/log_alpha"])
    errs["post/log_alpha"] = parity.rel_err(a[0:1], g["s0/post/log_alpha"])
    return errs


@pytest.mark.parametrize("name", ["sac_humanoid_mid", "sac_humanoid_b4096_mid"])
def test_sac_mid_state_step_matches_reference_golden(name):
    """One step from a mid-training state (fixtures_lib.mid_state: Adam moments
    after t = 7 steps, log-alpha off its init), restored through the
    reference-format snapshot (restore_from_snapshot), at 1e-5 against the
    reference's own step and against the oracle on the same state."""
    from fixtures_lib import mid_state, sac_params
    meta, g = parity.load(name)
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"],
                        pi_init_w=meta["pi_init_w"], q_init_w=meta["q_init_w"])
    ms = mid_state(params, ("policy", "qf1", "qf2"), meta["mid_state"]["t"],
                   meta["mid_state"]["seed"])
    tr = sac_trainer_for(meta)
    t = ms["t"]
    sd = lambda grp: {k: torch.from_numpy(v.copy()) for k, v in params[grp].items()}
    tr.restore_from_snapshot(dict(
        policy_state_dict=sd("policy"), policy_optim_state_dict=_optim_sd(tr.policy, ms["policy"], t),
        qf1_state_dict=sd("qf1"), qf1_optim_state_dict=_optim_sd(tr.qf1, ms["qf1"], t),
        target_qf1_state_dict=sd("target_qf1"),
        qf2_state_dict=sd("qf2"), qf2_optim_state_dict=_optim_sd(tr.qf2, ms["qf2"], t),
        target_qf2_state_dict=sd("target_qf2"),
        log_alpha=torch.tensor([float(ms["log_alpha"])]), alpha_optim_state_dict=_alpha_sd(ms),
        eval_statistics={}, _n_train_steps_total=t, _need_to_update_eval_statistics=True))
    orc = sac_oracle_from_gpu(tr, meta)
    batch = batch_from(meta, g["s0/idx"])
    tr.train_from_torch(batch, eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    torch.cuda.synchronize()
    out = orc.step(so.NumpyReplay.to_torch(batch), g["s0/eps1"], g["s0/eps2"])
    groups = (("policy", tr.policy, PARAM_ORDER_POLICY), ("qf1", tr.qf1, PARAM_ORDER_Q),
              ("qf2", tr.qf2, PARAM_ORDER_Q))
    errs = _golden_errors(g, tr, groups, meta)
    for grp, mod in (("policy", tr.policy), ("qf1", tr.qf1), ("qf2", tr.qf2),
                     ("target_qf1", tr.target_qf1), ("target_qf2", tr.target_qf2)):
        for pn, tt in mod.state_dict().items():
            errs[f"post/{grp}/{pn}"] = parity.compare(g, f"s0/post/{grp}/{pn}", tt.cpu().numpy())
    st = tr.get_diagnostics()
    for k in ("QF1 Loss", "QF2 Loss", "Policy Loss", "Alpha", "Alpha Loss", "Log Pis Mean"):
        errs[f"stat/{k}"] = parity.stat_err(st[k], g, f"s0/stat/{k}")
    # and the oracle on the same state (whole tensors)
    for grp, mod, order in groups:
        gv = module_tensors(tr, mod, tr.grads)
        for pn in order:
            errs[f"oracle/grad/{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(),
                                                             out["grads"][grp][pn].numpy())
    _check(errs, {}, name, 0)


def test_particle_mid_state_step_matches_reference_golden():
    """BASELINE configs[4] (K=10 shared-head critic, Ant-v2 dims, B=4096): one
    step from a mid-training state at 1e-5 against the reference's step."""
    from fixtures_lib import mid_state, sac_params
    from test_gpu_particle import particle_trainer_for
    meta, g = parity.load("poac_ant_b4096_mid")
    K = meta["K"]
    params = sac_params(meta["obs_dim"], meta["act_dim"], meta["hidden"], meta["seed"], q_out=K,
                        q_last_bias=np.linspace(meta["q_min"], meta["q_max"], K),
                        pi_init_w=meta["pi_init_w"])
    ms = mid_state(params, ("policy", "qf1"), meta["mid_state"]["t"], meta["mid_state"]["seed"])
    tr = particle_trainer_for(meta)
    t = ms["t"]
    sd = lambda grp: {k: torch.from_numpy(v.copy()) for k, v in params[grp].items()}
    tr.restore_from_snapshot(dict(
        policy_state_dict=sd("policy"),
        policy_optim_state_dict=_optim_sd(tr.policy, ms["policy"], t),
        qfs_state_dicts=[sd("qf1")], qfs_optims_state_dicts=[_optim_sd(tr.qfs[0], ms["qf1"], t)],
        target_qfs_state_dicts=[sd("target_qf1")],
        log_alpha=torch.tensor([float(ms["log_alpha"])]), alpha_optim_state_dict=_alpha_sd(ms),
        eval_statistics={}, _n_train_steps_total=t, _need_to_update_eval_statistics=True))
    orc = poac_oracle_from_gpu(tr, meta)
    batch = batch_from(meta, g["s0/idx"])
    tr.train_from_torch(batch, eps1=g["s0/eps1"], eps2=g["s0/eps2"])
    torch.cuda.synchronize()
    out = orc.step(so.NumpyReplay.to_torch(batch), g["s0/eps1"], g["s0/eps2"])
    groups = (("policy", tr.policy, PARAM_ORDER_POLICY), ("qf", tr.qfs[0], PARAM_ORDER_Q))
    errs = _golden_errors(g, tr, groups, meta)
    for grp, mod in (("policy", tr.policy), ("qf", tr.qfs[0]), ("tf", tr.tfs[0])):
        for pn, tt in mod.state_dict().items():
            errs[f"post/{grp}/{pn}"] = parity.compare(g, f"s0/post/{grp}/{pn}", tt.cpu().numpy())
    st = tr.get_diagnostics()
    for i in range(K):
        errs[f"stat/QF{i} Loss"] = parity.stat_err(st[f"QF{i} Loss"], g, f"s0/stat/QF{i} Loss")
    for grp, mod, order in groups:
        gv = module_tensors(tr, mod, tr.grads)
        for pn in order:
            errs[f"oracle/grad/{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(),
                                                             out["grads"][grp][pn].numpy())
    _check(errs, {}, "poac_ant_b4096_mid", 0)
