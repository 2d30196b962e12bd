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
