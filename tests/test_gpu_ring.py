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
