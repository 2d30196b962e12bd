"""Ragged shapes on the GPU, every trainer kind against the fp32 CPU oracle:
batch sizes that are not tile multiples (1, 37, 300, and 1029 / 1100 on the
large-batch kernels: the LDS-DMA pipelined forward and backward products with
partial tiles and partial K stages, split-K chunks that end mid stage),
hidden widths that are not multiples of the 32- or 64-wide tiles (48, 80),
odd observation / action widths.
One step from identical state; every gradient tensor within 1e-5
(norm-relative) of the oracle's."""
import numpy as np
import pytest
import torch

import parity
from fixtures_lib import (PARAM_ORDER_POLICY, PARAM_ORDER_Q, goac_params, ptrain_params,
                          sac_params, synthetic_transitions)
from gpu_helpers import Space, module_tensors, producers

pytestmark = pytest.mark.gpu

SHAPES = [(11, 3, 32, 1), (11, 3, 32, 37), (7, 5, 48, 300), (376, 17, 256, 37),
          (7, 5, 48, 1100), (13, 6, 80, 1029)]


def _batch(Do, Da, B, seed):
    data = synthetic_transitions(max(4 * B, 64), Do, Da, seed=seed)
    idx = np.random.RandomState(seed).randint(0, len(data["rewards"]), B)
    return {k: v[idx] for k, v in data.items()}


def _compare(tr, groups, want):
    worst = {}
    for grp, mod, order in groups:
        gv = module_tensors(tr, mod, tr.grads)
        for pn in order:
            worst[f"{grp}/{pn}"] = parity.rel_err(gv[pn].cpu().numpy(), want[grp][pn].numpy())
    bad = {k: v for k, v in worst.items() if v > 1e-5}
    assert not bad, bad


@pytest.mark.parametrize("Do,Da,H,B", SHAPES)
def test_sac_ragged(Do, Da, H, B):
    _sac_case(Do, Da, H, B)


# large batch with B a multiple of 256 and hidden % 32 == 0: the critics'
# last-layer dW is written as split-K slabs by the targets kernel
# (critic_targets_kernel, rows.hip; 2-8 row blocks x 2-8 column groups)
@pytest.mark.parametrize("Do,Da,H,B", [(11, 3, 64, 1024), (7, 5, 96, 2048), (376, 17, 256, 1024)])
def test_sac_last_layer_slabs_in_targets(Do, Da, H, B):
    _sac_case(Do, Da, H, B)


def _sac_case(Do, Da, H, B):
    from oac_amd import SACTrainer
    from oracle import sac_oracle as so
    params = sac_params(Do, Da, [H, H], 3, pi_init_w=0.2, q_init_w=0.1)
    pp, qp = producers(params)
    tr = SACTrainer(pp, qp, action_space=Space(Da), policy_lr=3e-4, qf_lr=3e-4,
                    soft_target_tau=5e-3, use_automatic_entropy_tuning=True)
    b = _batch(Do, Da, B, 1)
    rs = np.random.RandomState(2)
    e1 = rs.standard_normal((B, Da)).astype(np.float32)
    e2 = rs.standard_normal((B, Da)).astype(np.float32)
    tr.train_from_torch(b, eps1=e1, eps2=e2)
    torch.cuda.synchronize()
    out = so.SACOracle(params, Do, Da, policy_lr=3e-4, qf_lr=3e-4).step(b, e1, e2)
    _compare(tr, [("policy", tr.policy, PARAM_ORDER_POLICY), ("qf1", tr.qf1, PARAM_ORDER_Q),
                  ("qf2", tr.qf2, PARAM_ORDER_Q)], out["grads"])


@pytest.mark.parametrize("Do,Da,H,B", SHAPES)
def test_particle_oac_ragged(Do, Da, H, B):
    from oac_amd import ParticleTrainerOAC
    from oracle import sac_oracle as so
    K = 7
    params = sac_params(Do, Da, [H, H], 3, q_out=K, pi_init_w=0.2, q_init_w=0.1,
                        q_last_bias=np.linspace(0.0, 30.0, K))
    pp, qp = producers(params, q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                       "target_qf1"))
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), policy_lr=3e-4,
                            qf_lr=3e-4, soft_target_tau=5e-3, use_automatic_entropy_tuning=True,
                            deterministic=False, q_min=0.0, q_max=30.0, share_layers=True)
    b = _batch(Do, Da, B, 4)
    rs = np.random.RandomState(5)
    e1 = rs.standard_normal((B, Da)).astype(np.float32)
    e2 = rs.standard_normal((B, Da)).astype(np.float32)
    tr.train_from_torch(b, eps1=e1, eps2=e2)
    torch.cuda.synchronize()
    out = so.ParticleOACOracle(params, Do, Da, K, policy_lr=3e-4, qf_lr=3e-4).step(b, e1, e2)
    _compare(tr, [("policy", tr.policy, PARAM_ORDER_POLICY), ("qf", tr.qfs[0], PARAM_ORDER_Q)],
             out["grads"])


@pytest.mark.parametrize("Do,Da,H,B", SHAPES)
def test_goac_ragged(Do, Da, H, B):
    from test_gpu_goac import goac_producers
    from oac_amd import GaussianTrainer
    from oracle import sac_oracle as so
    params = goac_params(Do, Da, [H, H], 3, 0.0, 100.0, pi_init_w=0.2, q_init_w=0.1)
    pp, qp = goac_producers(params)
    tr = GaussianTrainer(pp, qp, action_space=Space(Da), policy_lr=3e-4, qf_lr=3e-4,
                         soft_target_tau=5e-3, q_min=0.0, q_max=100.0, share_layers=True,
                         counts=True)
    b = _batch(Do, Da, B, 6)
    b["counts"] = np.random.RandomState(7).randint(0, 2, (B, 1)).astype(np.float64)
    tr.train_from_torch(b)
    torch.cuda.synchronize()
    out = so.GaussianOACOracle(params, Do, Da, q_min=0.0, q_max=100.0, policy_lr=3e-4,
                               qf_lr=3e-4).step(b)
    _compare(tr, [("policy", tr.policy, PARAM_ORDER_POLICY[:6]),
                  ("target_policy", tr.target_policy, PARAM_ORDER_POLICY[:6]),
                  ("qf", tr.q, PARAM_ORDER_Q)], out["grads"])


@pytest.mark.parametrize("Do,Da,H,B", SHAPES)
def test_ptrain_ragged(Do, Da, H, B):
    from test_gpu_ptrain import ptrain_producers
    from oac_amd import ParticleTrainer
    from oracle import sac_oracle as so
    K = 10
    params = ptrain_params(Do, Da, [H, H], 3, K, 0.0, 50.0, pi_init_w=0.2, q_init_w=0.1)
    pp, qp = ptrain_producers(params)
    tr = ParticleTrainer(pp, qp, n_estimators=K, action_space=Space(Da), policy_lr=3e-4,
                         qf_lr=3e-4, soft_target_tau=5e-3, q_min=0.0, q_max=50.0,
                         share_layers=True, counts=True)
    b = _batch(Do, Da, B, 8)
    b["counts"] = np.random.RandomState(9).randint(0, 2, (B, 1)).astype(np.float64)
    tr.train_from_torch(b)
    torch.cuda.synchronize()
    out = so.ParticleUBOracle(params, Do, Da, K, tr.delta_index, q_min=0.0, q_max=50.0,
                              policy_lr=3e-4, qf_lr=3e-4).step(b)
    _compare(tr, [("policy", tr.policy, PARAM_ORDER_POLICY[:6]),
                  ("target_policy", tr.target_policy, PARAM_ORDER_POLICY[:6]),
                  ("qf", tr.qfs[0], PARAM_ORDER_Q)], out["grads"])
