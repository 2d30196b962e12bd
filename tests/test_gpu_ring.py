"""Device-resident ring path (SACTrainer.train_from_ring): the minibatches of
up to 8 consecutive steps are gathered by one launch at the start of an
n-step graph (csrc/sac_plan.hip, gather_steps); the result must not depend on
how the steps are split into calls -- one call of 16 steps (two batched
gathers), two calls of 8, sixteen calls of 1 are bitwise equal."""
import numpy as np
import pytest
import torch

from fixtures_lib import sac_params, synthetic_transitions

pytestmark = pytest.mark.gpu

Do, Da, H, B = 11, 3, 32, 32


def _trainer():
    from gpu_helpers import producers, Space
    from oac_amd import SACTrainer
    pp, qp = producers(sac_params(Do, Da, [H, H], 3, pi_init_w=0.2, q_init_w=0.1))
    return SACTrainer(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0,
                      policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3,
                      use_automatic_entropy_tuning=True)


def _run(splits):
    from oac_amd import DeviceIndexStream, ReplayBuffer
    from gpu_helpers import Space
    rb = ReplayBuffer(2000, Space(Do), Space(Da), device="cuda:0")
    data = synthetic_transitions(2000, Do, Da, seed=1)
    rb.load_transitions(torch.from_numpy(rb._rows_from(
        data["observations"], data["actions"], data["rewards"], data["next_observations"],
        data["terminals"])).cuda())
    st = DeviceIndexStream(rb, B, chunk=16, seed=4)
    tr = _trainer()
    for n in splits:
        st.before_step(n)
        tr.train_from_ring(rb._storage, st.ring, st.slots, B, n_steps=n)
    torch.cuda.synchronize()
    return torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy()


def test_ring_steps_independent_of_call_split():
    a = _run([16])
    b = _run([8, 8])
    c = _run([1] * 16)
    assert np.isfinite(a).all()
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, c)


@pytest.mark.parametrize("prefetch", [0, 1])
def test_ring_direct_rows_equal_the_gather_launch_path(prefetch):
    """The small-batch ring step's default form -- layer 0 reading its rows
    through the device index ring, side blocks copying the batch and drawing
    eps (the drop-in step's form) -- against the gather launch per 8 steps
    (tuning ring_direct=-1), with and without the next step's critic forward
    inside the policy backward (ring_prefetch): bitwise equal states.  The
    prefetch form keeps the policy-head dX in a launch of its own (its own
    summation order), so its direct-rows counterpart is run that way too
    (head_dh2=-1)."""
    from oac_amd import _lib
    try:
        _lib.set_tuning(head_dh2=-1 if prefetch else 0)
        a = _run([16, 8, 4, 2, 1, 1])
        _lib.set_tuning(ring_direct=-1, ring_prefetch=prefetch)
        b = _run([16, 8, 4, 2, 1, 1])
    finally:
        _lib.set_tuning(ring_direct=0, ring_prefetch=0, head_dh2=0)
    assert np.isfinite(a).all()
    np.testing.assert_array_equal(a, b)


# ------------------------------------------- counts=True trainers on the ring
def _counts_trainer(kind):
    from fixtures_lib import goac_params, ptrain_params
    from gpu_helpers import producers, Space
    if kind == "goac":
        from oac_amd import GaussianTrainer
        from test_gpu_goac import goac_producers
        pp, qp = goac_producers(goac_params(Do, Da, [H, H], 3, 0.0, 100.0, pi_init_w=0.2,
                                            q_init_w=0.1))
        return GaussianTrainer(pp, qp, action_space=Space(Da), policy_lr=1e-3, qf_lr=1e-3,
                               soft_target_tau=5e-3, q_min=0.0, q_max=100.0, share_layers=True,
                               counts=True)
    if kind == "ptrain":
        from oac_amd import ParticleTrainer
        from test_gpu_ptrain import ptrain_producers
        pp, qp = ptrain_producers(ptrain_params(Do, Da, [H, H], 3, 5, 0.0, 50.0, pi_init_w=0.2,
                                                q_init_w=0.1))
        return ParticleTrainer(pp, qp, n_estimators=5, action_space=Space(Da), policy_lr=1e-3,
                               qf_lr=1e-3, soft_target_tau=5e-3, q_min=0.0, q_max=50.0,
                               share_layers=True, counts=True)
    from oac_amd import ParticleTrainerOAC
    K = 5
    pp, qp = producers(sac_params(Do, Da, [H, H], 3, q_out=K, pi_init_w=0.2,
                                  q_last_bias=np.linspace(0.0, 50.0, K)),
                       q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1", "target_qf1"))
    return ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), policy_lr=1e-3,
                              qf_lr=1e-3, soft_target_tau=5e-3, use_automatic_entropy_tuning=True,
                              deterministic=False, q_min=0.0, q_max=50.0, share_layers=True,
                              counts=True)


def _count_buffer():
    from oac_amd import ReplayBufferCount
    from gpu_helpers import Space
    rb = ReplayBufferCount(300, Space(Do), Space(Da), device="cuda:0", index_source="device")
    data = synthetic_transitions(300, Do, Da, seed=1)
    rb.load_transitions(torch.from_numpy(rb._rows_from(
        data["observations"], data["actions"], data["rewards"], data["next_observations"],
        data["terminals"])).cuda())
    return rb


@pytest.mark.parametrize("kind", ["goac", "ptrain", "poac"])
def test_counts_ring_equals_random_batch_path(kind):
    """counts=True trainers from the device index ring (counts read and bumped
    inside the step's graph) equal the ReplayBufferCount.random_batch path
    (host-driven draw + counts update, then train) on the same index stream:
    parameters bitwise, counts array equal.  A small buffer (300 rows, B=32)
    so rows repeat within and across batches."""
    from oac_amd import DeviceIndexStream
    steps, seed = 16, 4
    # host path
    rb_a = _count_buffer()
    rb_a.seed_device_stream(seed)
    tr_a = _counts_trainer(kind)
    for _ in range(steps):
        tr_a.train(rb_a.random_batch(B))
    # ring path: two graph launches of 8 steps
    rb_b = _count_buffer()
    st = DeviceIndexStream(rb_b, B, chunk=8, seed=seed)
    tr_b = _counts_trainer(kind)
    for _ in range(2):
        st.before_step(8)
        tr_b.train_from_ring(rb_b._storage, st.ring, st.slots, B, n_steps=8,
                             count_state=rb_b.device_count_state())
    torch.cuda.synchronize()
    assert torch.equal(rb_a._counts, rb_b._counts)
    assert int(rb_a._counts.sum()) > 0
    for name in ("params", "targets", "adam_m", "adam_v"):
        np.testing.assert_array_equal(getattr(tr_a, name).cpu().numpy(),
                                      getattr(tr_b, name).cpu().numpy())
