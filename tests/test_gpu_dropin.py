"""The drop-in call pattern of rl_algorithm.py:160-167 -- np.random.randint
indices from ReplayBuffer.random_batch, then trainer.train(batch) once per
step -- on the asynchronous host-index path (pinned staging ring + one-step
graph on the current stream, oac_sac_step_host_idx) must equal the
synchronous device-index path bit for bit, across staging-ring wrap-around
and when mixed with the other step paths."""
import numpy as np
import pytest
import torch

from fixtures_lib import sac_params, synthetic_transitions
from gpu_helpers import Space, producers

pytestmark = pytest.mark.gpu

Do, Da, H, B, N = 11, 3, [32, 32], 16, 700


def _setup(dropin):
    from oac_amd import ReplayBuffer, SACTrainer
    pp, qp = producers(sac_params(Do, Da, H, 3, pi_init_w=0.2, q_init_w=0.1))
    tr = SACTrainer(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0,
                    policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3, device="cuda:0", seed=7)
    tr._no_dropin = not dropin
    rb = ReplayBuffer(N, Space(Do), Space(Da), device="cuda:0")
    d = synthetic_transitions(N, Do, Da, seed=1)
    rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                       rewards=d["rewards"], next_observations=d["next_observations"],
                       terminals=d["terminals"])])
    return tr, rb


def _state(tr):
    torch.cuda.synchronize()
    return torch.cat([tr.params, tr.targets, tr.alpha_state[:4]]).cpu().numpy()


def _loop(tr, rb, steps, seed=1):
    np.random.seed(seed)
    for _ in range(steps):
        batch = rb.random_batch(B)
        batch["buffer"] = rb            # rl_algorithm.py:166
        tr.train(batch)


def test_dropin_equals_device_index_path_across_ring_wrap():
    # 300 steps: more than two passes over the 128-slot staging ring
    a, ra = _setup(True)
    b, rb = _setup(False)
    _loop(a, ra, 300)
    _loop(b, rb, 300)
    assert a._n_train_steps_total == b._n_train_steps_total == 300
    assert np.array_equal(_state(a), _state(b))
    assert int(a.step_state[1].item()) == 300


def test_dropin_mixed_with_other_paths_keeps_the_batch_counter():
    from oac_amd import DeviceIndexStream
    a, ra = _setup(True)
    b, rb = _setup(False)
    for tr, r in ((a, ra), (b, rb)):
        _loop(tr, r, 5, seed=2)
        st = DeviceIndexStream(r, B, chunk=8, seed=4)   # ring path in between
        st.before_step(4)
        tr.train_from_ring(r._storage, st.ring, st.slots, B, n_steps=4)
        d = synthetic_transitions(N, Do, Da, seed=1)
        idx = np.arange(B) * 3
        tr.train_from_torch({k: v[idx] for k, v in d.items()})   # host batch path
        tr.end_epoch(0)                                          # stats on the next step
        _loop(tr, r, 7, seed=3)
    assert np.array_equal(_state(a), _state(b))
    assert a.get_diagnostics().keys() == b.get_diagnostics().keys()
    for k in a.get_diagnostics():
        assert a.get_diagnostics()[k] == b.get_diagnostics()[k], k


def test_dropin_rejects_out_of_range_indices():
    from oac_amd.replay_buffer import DeviceBatch
    a, ra = _setup(True)
    bad = DeviceBatch(ra, host_indices=np.full(B, N + 5, dtype=np.int64))
    with pytest.raises(RuntimeError, match="outside the replay"):
        a.train(bad)


# ------------------------------------------------ host-read index ring
# The drop-in step of the large-batch SAC plan and of the particle / g-oac
# trainers reads its indices straight from the pinned host ring in the gather
# launch (oac_sac_step_host_idx, PlanBase::idx_host): no H2D copy before the
# step graph.  It must equal the device-index path bit for bit across the
# staging ring's wrap-around.
def _kind_trainer(kind, dropin):
    from fixtures_lib import goac_params
    from gpu_helpers import producers, Space
    # hidden 64 at B=1024: the direct large-batch gather (layer-0 tiles read the
    # replay rows through the index slot, side workgroups draw eps and copy the
    # batch -- sac_plan.h big_direct_ok); hidden 32 keeps the gather launch
    Hh = 64 if kind.endswith("_direct") else 32
    kind = kind.replace("_direct", "")
    if kind == "sac_large":
        from oac_amd import SACTrainer
        pp, qp = producers(sac_params(Do, Da, [Hh, Hh], 3, pi_init_w=0.2, q_init_w=0.1))
        tr = SACTrainer(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0,
                        policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3, device="cuda:0", seed=7)
    elif kind == "goac":
        from oac_amd import GaussianTrainer
        from test_gpu_goac import goac_producers
        pp, qp = goac_producers(goac_params(Do, Da, [Hh, Hh], 3, 0.0, 100.0, pi_init_w=0.2,
                                            q_init_w=0.1))
        tr = GaussianTrainer(pp, qp, action_space=Space(Da), policy_lr=1e-3, qf_lr=1e-3,
                             soft_target_tau=5e-3, q_min=0.0, q_max=100.0, share_layers=True)
    else:
        from oac_amd import ParticleTrainerOAC
        K = 5
        pp, qp = producers(sac_params(Do, Da, [Hh, Hh], 3, q_out=K, pi_init_w=0.2,
                                      q_last_bias=np.linspace(0.0, 50.0, K)),
                           q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1", "target_qf1"))
        tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), policy_lr=1e-3,
                                qf_lr=1e-3, soft_target_tau=5e-3, use_automatic_entropy_tuning=True,
                                deterministic=False, q_min=0.0, q_max=50.0, share_layers=True)
    tr._no_dropin = not dropin
    return tr


@pytest.mark.parametrize("kind", ["sac_large", "sac_large_direct", "poac", "poac_direct", "goac"])
def test_host_read_dropin_equals_device_index_path(kind):
    from oac_amd import ReplayBuffer
    from gpu_helpers import Space
    Bk, Nk, steps = (1024, 3000, 136) if kind.startswith("sac_large") or kind.endswith("_direct") \
        else (B, N, 140)

    def run(dropin):
        tr = _kind_trainer(kind, dropin)
        rb = ReplayBuffer(Nk, Space(Do), Space(Da), device="cuda:0")
        d = synthetic_transitions(Nk, Do, Da, seed=1)
        rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                           rewards=d["rewards"], next_observations=d["next_observations"],
                           terminals=d["terminals"])])
        np.random.seed(3)
        for _ in range(steps):
            batch = rb.random_batch(Bk)
            batch["buffer"] = rb
            tr.train(batch)
        return tr
    a, b = run(True), run(False)
    assert a._n_train_steps_total == b._n_train_steps_total == steps
    sa, sb = _state(a), _state(b)
    assert np.isfinite(sa).all()
    assert np.array_equal(sa, sb)


def test_host_read_dropin_mixed_paths_across_ring_wrap():
    """The large-batch drop-in step (host-read index ring) interleaved with the
    device-ring path: each ring call advances the batch counter by 3, so the
    following drop-in steps start mid-chunk and the staging ring wraps (more
    than 128 staged slots).  A slot must never be rewritten while a queued step
    still reads it: bitwise equal to the device-index path."""
    from oac_amd import DeviceIndexStream, ReplayBuffer
    from gpu_helpers import Space
    Bk, Nk = 1024, 3000

    def run(dropin):
        tr = _kind_trainer("sac_large", dropin)
        rb = ReplayBuffer(Nk, Space(Do), Space(Da), device="cuda:0")
        d = synthetic_transitions(Nk, Do, Da, seed=1)
        rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                           rewards=d["rewards"], next_observations=d["next_observations"],
                           terminals=d["terminals"])])
        np.random.seed(5)
        for seg, n in enumerate((37, 61, 45, 50)):
            for _ in range(n):
                batch = rb.random_batch(Bk)
                batch["buffer"] = rb
                tr.train(batch)
            st = DeviceIndexStream(rb, Bk, chunk=3, seed=4 + seg)
            st.before_step(3)
            tr.train_from_ring(rb._storage, st.ring, st.slots, Bk, n_steps=3)
        return tr
    a, b = run(True), run(False)
    assert a._n_train_steps_total == b._n_train_steps_total == 193 + 12
    sa, sb = _state(a), _state(b)
    assert np.isfinite(sa).all()
    assert np.array_equal(sa, sb)


def test_eager_phase_calls_keep_launch_records_bounded():
    """oac_sac_step_phase (the torch-transport data-parallel path) at a
    large batch: every step's launches reuse their device launch records
    (kernels.h BatchCache, keyed by the launch's index within one step), so
    100 eager steps add no records after the first and the positions stay
    those of one step."""
    import ctypes
    from oac_amd import SACTrainer, _lib
    Bb = 1024
    pp, qp = producers(sac_params(Do, Da, [64, 64], 3, pi_init_w=0.2, q_init_w=0.1))
    tr = SACTrainer(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0,
                    policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3, device="cuda:0", seed=7)
    d = synthetic_transitions(Bb, Do, Da, seed=1)
    tr.train_from_torch(d)   # the plan, with this batch and Philox eps in its workspace
    torch.cuda.synchronize()
    plan = tr._last_plan
    L = _lib.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    st = (ctypes.c_int64 * 4)()

    def stats():
        _lib.check(L.oac_sac_cache_stats(plan.handle, st))
        return list(st)

    def step():
        for ph in (0, 1, 2, 3):
            _lib.check(L.oac_sac_step_phase(plan.handle, ph, _lib.OAC_STEP_DEVICE_EPS, sp))

    step()
    torch.cuda.synchronize()
    used0, pos0, _, _ = stats()
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    used, pos, hits, misses = stats()
    print("launch records: used %d positions %d hits %d misses %d" % (used, pos, hits, misses))
    assert used == used0 and pos == pos0 and 0 < pos <= 32 and used <= 64
    assert torch.isfinite(tr.params).all()
