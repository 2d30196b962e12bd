"""Checkpoint format (trainer/trainer.py:299-369): a run
resumes across the reference and this build.

* A checkpoint the reference's own SACTrainer wrote (tests/golden/
  sac_snapshot.pt, make_golden.py gen_sac_snapshot -- torch.save of
  get_snapshot() after two steps) restores into oac_amd.SACTrainer, whose
  get_snapshot() then returns the same keys, tensors and Adam state layout,
  and whose next step equals the reference's next step.
* oac_amd's own checkpoint survives torch.save / torch.load(weights_only=True)
  and resumes bitwise: restored trainer == uninterrupted trainer."""
import io
import os

import numpy as np
import pytest
import torch

import parity
from fixtures_lib import PARAM_ORDER_POLICY, PARAM_ORDER_Q, sac_params
from gpu_helpers import batch_from, sac_trainer_for

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture():
    return torch.load(os.path.join(HERE, "golden", "sac_snapshot.pt"), weights_only=True)


def _trainer(meta):
    m = dict(obs_dim=meta["obs_dim"], act_dim=meta["act_dim"], hidden=meta["hidden"],
             discount=0.99, reward_scale=1.0, lr=meta["lr"], tau=meta["tau"], auto_alpha=True,
             log_alpha0=0.0, seed=meta["seed"], pi_init_w=meta["pi_init_w"],
             q_init_w=meta["q_init_w"])
    return sac_trainer_for(m), m


def _cpu(x):
    return x.detach().cpu() if torch.is_tensor(x) else torch.as_tensor(x)


def test_reference_checkpoint_restores_and_resumes():
    fx = _fixture()
    meta, ref = fx["meta"], fx["snapshot"]
    tr, m = _trainer(meta)
    tr.restore_from_snapshot(ref)
    ours = tr.get_snapshot()
    assert set(ours) == set(ref)
    assert ours["_n_train_steps_total"] == ref["_n_train_steps_total"] == 2
    for key in ("policy_state_dict", "qf1_state_dict", "qf2_state_dict", "target_qf1_state_dict",
                "target_qf2_state_dict"):
        assert list(ours[key]) == list(ref[key]), key
        for k, v in ref[key].items():
            torch.testing.assert_close(_cpu(ours[key][k]), v, rtol=0, atol=0)
    for key in ("policy_optim_state_dict", "qf1_optim_state_dict", "qf2_optim_state_dict",
                "alpha_optim_state_dict"):
        so, sr = ours[key]["state"], ref[key]["state"]
        assert sorted(so) == sorted(sr), key
        for i in sr:
            assert int(so[i]["step"]) == int(sr[i]["step"])
            for f in ("exp_avg", "exp_avg_sq"):
                torch.testing.assert_close(_cpu(so[i][f]).reshape(sr[i][f].shape), sr[i][f],
                                           rtol=0, atol=0)
        for f in ("lr", "betas", "eps"):
            assert ours[key]["param_groups"][0][f] == ref[key]["param_groups"][0][f]
    torch.testing.assert_close(_cpu(ours["log_alpha"]).reshape(1), ref["log_alpha"].reshape(1),
                               rtol=0, atol=0)
    # the reference's third step from this checkpoint
    s3 = fx["step3"]
    meta_b = dict(m, n_replay=meta["n_replay"])
    tr.train_from_torch(batch_from(meta_b, s3["idx"].numpy()), eps1=s3["eps1"].numpy(),
                        eps2=s3["eps2"].numpy())
    torch.cuda.synchronize()
    worst = 0.0
    for g in ("policy", "qf1", "qf2", "target_qf1", "target_qf2"):
        sd = getattr(tr, g).state_dict()
        for k, v in s3["post"][g].items():
            worst = max(worst, parity.rel_err(_cpu(sd[k]).numpy(), v.numpy()))
    assert worst < 1e-5, worst
    assert parity.rel_err(tr.log_alpha.detach().cpu().numpy(), s3["log_alpha"].numpy()) < 1e-5


def test_own_checkpoint_roundtrip_resumes_bitwise():
    fx = _fixture()
    meta = fx["meta"]
    a, m = _trainer(meta)
    meta_b = dict(m, n_replay=300)

    def step(tr, s):
        r = np.random.RandomState(100 + s)
        idx = r.randint(0, 300, meta["B"])
        e1 = r.standard_normal((meta["B"], meta["act_dim"])).astype(np.float32)
        e2 = r.standard_normal((meta["B"], meta["act_dim"])).astype(np.float32)
        tr.train_from_torch(batch_from(meta_b, idx), eps1=e1, eps2=e2)

    for s in range(3):
        step(a, s)
    buf = io.BytesIO()
    torch.save(a.get_snapshot(), buf)
    buf.seek(0)
    ss = torch.load(buf, weights_only=True)
    b, _ = _trainer(meta)
    b.restore_from_snapshot(ss)
    for s in range(3, 5):
        step(a, s)
        step(b, s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.params.cpu().numpy(), b.params.cpu().numpy())
    np.testing.assert_array_equal(a.targets.cpu().numpy(), b.targets.cpu().numpy())
    np.testing.assert_array_equal(a.adam_m.cpu().numpy(), b.adam_m.cpu().numpy())


# ------------------------------------------ g-oac / p-oac (target_policy) trainers
def _det_trainer(kind):
    fx = torch.load(os.path.join(HERE, "golden", f"{kind}_snapshot.pt"), weights_only=True)
    meta = dict(fx["meta"], counts=True, soft=None)
    if kind == "goac":
        from test_gpu_goac import goac_trainer_for
        tr = goac_trainer_for(meta)
        mods = dict(policy=tr.policy, target_policy=tr.target_policy, qf=tr.q, tf=tr.q_target)
    else:
        from test_gpu_ptrain import ptrain_trainer_for
        tr = ptrain_trainer_for(meta)
        mods = dict(policy=tr.policy, target_policy=tr.target_policy, qf=tr.qfs[0],
                    tf=tr.tfs[0])
    return fx, meta, tr, mods


@pytest.mark.parametrize("kind", ["goac", "ptrain"])
def test_det_reference_checkpoint_restores_and_resumes(kind):
    """A checkpoint the reference's GaussianTrainer / particle_trainer
    ParticleTrainer wrote (make_golden.py gen_det_snapshot) restores into the
    oac_amd trainer with the same keys, tensors and Adam state layout (no
    state for the never-updated log-std heads), and the next step matches the
    reference's."""
    fx, meta, tr, mods = _det_trainer(kind)
    ref = fx["snapshot"]
    tr.restore_from_snapshot(ref)
    ours = tr.get_snapshot()
    assert set(ours) == set(ref)
    for key in ("policy_state_dict", "target_policy_state_dict"):
        for k, v in ref[key].items():
            torch.testing.assert_close(_cpu(ours[key][k]), v, rtol=0, atol=0)
    for key in ("qfs_state_dicts", "target_qfs_state_dicts"):
        assert len(ours[key]) == len(ref[key]) == 1
        for k, v in ref[key][0].items():
            torch.testing.assert_close(_cpu(ours[key][0][k]), v, rtol=0, atol=0)
    for so, sr in ((ours["policy_optim_state_dict"], ref["policy_optim_state_dict"]),
                   (ours["target_policy_opt_state_dict"], ref["target_policy_opt_state_dict"]),
                   (ours["qfs_optims_state_dicts"][0], ref["qfs_optims_state_dicts"][0])):
        assert sorted(so["state"]) == sorted(sr["state"])
        for i in sr["state"]:
            assert int(so["state"][i]["step"]) == int(sr["state"][i]["step"])
            for f in ("exp_avg", "exp_avg_sq"):
                torch.testing.assert_close(_cpu(so["state"][i][f]).reshape(sr["state"][i][f].shape),
                                           sr["state"][i][f], rtol=0, atol=0)
    s3 = fx["step3"]
    b = batch_from(meta, s3["idx"].numpy())
    b["counts"] = s3["counts"].numpy()
    tr.train_from_torch(b)
    torch.cuda.synchronize()
    worst = 0.0
    for g, mod in mods.items():
        sd = mod.state_dict()
        for k, v in s3["post"][g].items():
            worst = max(worst, parity.rel_err(_cpu(sd[k]).numpy(), v.numpy()))
    assert worst < 1e-5, worst


@pytest.mark.parametrize("kind", ["goac", "ptrain"])
def test_det_own_checkpoint_roundtrip_resumes_bitwise(kind):
    fx, meta, a, _ = _det_trainer(kind)
    meta_b = dict(meta, n_replay=300)

    def step(tr, s):
        r = np.random.RandomState(200 + s)
        b = batch_from(meta_b, r.randint(0, 300, meta["B"]))
        b["counts"] = (r.randint(0, 3, (meta["B"], 1)) * (r.uniform(0, 1, (meta["B"], 1)) < 0.5))
        tr.train_from_torch(b)

    for s in range(3):
        step(a, s)
    buf = io.BytesIO()
    torch.save(a.get_snapshot(), buf)
    buf.seek(0)
    ss = torch.load(buf, weights_only=True)
    _, _, b, _ = _det_trainer(kind)
    b.restore_from_snapshot(ss)
    for s in range(3, 5):
        step(a, s)
        step(b, s)
    torch.cuda.synchronize()
    for name in ("params", "targets", "adam_m", "adam_v"):
        np.testing.assert_array_equal(getattr(a, name).cpu().numpy(),
                                      getattr(b, name).cpu().numpy())
