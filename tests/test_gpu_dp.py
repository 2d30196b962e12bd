"""GPU data-parallel trainer: 2 ranks sharing cuda:0 (gloo transport -- RCCL
refuses two ranks on one device; the 8-GPU run uses RCCL) must equal the
single-process GPU trainer on the concatenated batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import parity
from fixtures_lib import sac_params, synthetic_transitions

pytestmark = pytest.mark.gpu

Do, Da, H, BL, STEPS = 11, 3, 32, 32, 3
META = dict(obs_dim=Do, act_dim=Da, hidden=[H, H], discount=0.99, reward_scale=1.0, lr=1e-3,
            tau=5e-3, auto_alpha=True, log_alpha0=0.0, seed=3, pi_init_w=0.2, q_init_w=0.1)


def _inputs(world):
    data = synthetic_transitions(500, Do, Da, seed=0)
    rs = np.random.RandomState(5)
    out = []
    for _ in range(STEPS):
        idx = rs.randint(0, 500, BL * world)
        e1 = rs.standard_normal((BL * world, Da)).astype(np.float32)
        e2 = rs.standard_normal((BL * world, Da)).astype(np.float32)
        out.append(({k: v[idx] for k, v in data.items()}, e1, e2))
    return out


def _trainer(dp, kind="sac"):
    from gpu_helpers import producers, Space
    if kind == "goac":
        from fixtures_lib import goac_params
        from oac_amd import GaussianTrainer
        from oac_amd.dp import DataParallelGaussianTrainer
        from test_gpu_goac import goac_producers
        pp, qp = goac_producers(goac_params(Do, Da, [H, H], 3, 0.0, 100.0, pi_init_w=0.2,
                                            q_init_w=0.1))
        cls = DataParallelGaussianTrainer if dp else GaussianTrainer
        return cls(pp, qp, action_space=Space(Da), discount=0.99, policy_lr=1e-3, qf_lr=1e-3,
                   soft_target_tau=5e-3, q_min=0.0, q_max=100.0, share_layers=True, counts=True)
    if kind == "ptrain":
        from fixtures_lib import ptrain_params
        from oac_amd import ParticleTrainer
        from oac_amd.dp import DataParallelParticleTrainer
        from test_gpu_ptrain import ptrain_producers
        pp, qp = ptrain_producers(ptrain_params(Do, Da, [H, H], 3, 5, 0.0, 50.0, pi_init_w=0.2,
                                                q_init_w=0.1))
        cls = DataParallelParticleTrainer if dp else ParticleTrainer
        return cls(pp, qp, n_estimators=5, action_space=Space(Da), discount=0.99,
                   policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3, q_min=0.0, q_max=50.0,
                   share_layers=True, counts=True)
    if kind == "poac":
        from oac_amd import ParticleTrainerOAC as ParticleTrainer
        from oac_amd.dp import DataParallelParticleTrainerOAC as DataParallelParticleTrainer
        K = 5
        pp, qp = producers(sac_params(Do, Da, [H, H], 3, q_out=K, pi_init_w=0.2,
                                      q_last_bias=np.linspace(0.0, 50.0, K)),
                           q_keys=("qf1", "qf2", "target_qf1", "target_qf2", "qf1",
                                   "target_qf1"))
        cls = DataParallelParticleTrainer if dp else ParticleTrainer
        return cls(pp, qp, n_estimators=K, action_space=Space(Da), discount=0.99,
                   policy_lr=1e-3, qf_lr=1e-3, soft_target_tau=5e-3,
                   use_automatic_entropy_tuning=True, deterministic=False, q_min=0.0,
                   q_max=50.0, share_layers=True, counts=True)
    from oac_amd import SACTrainer
    from oac_amd.dp import DataParallelSACTrainer
    pp, qp = producers(sac_params(Do, Da, [H, H], 3, pi_init_w=0.2, q_init_w=0.1))
    cls = DataParallelSACTrainer if dp else SACTrainer
    return cls(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0, policy_lr=1e-3,
               qf_lr=1e-3, soft_target_tau=5e-3, use_automatic_entropy_tuning=True)


def _with_counts(batch, step):
    b = dict(batch)
    rs = np.random.RandomState(100 + step)
    n = len(b["rewards"])
    b["counts"] = (rs.randint(0, 3, (n, 1)) * (rs.uniform(0, 1, (n, 1)) < 0.5)).astype(np.float64)
    return b


def _worker(rank, world, port, q, kind="sac"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = _trainer(True, kind)
    for step, (batch, e1, e2) in enumerate(_inputs(world)):
        sl = slice(rank * BL, (rank + 1) * BL)
        if kind in ("goac", "ptrain"):
            tr.train_from_torch({k: v[sl] for k, v in _with_counts(batch, step).items()})
            continue
        if kind == "poac":
            batch = _with_counts(batch, step)
        tr.train_from_torch({k: v[sl] for k, v in batch.items()}, eps1=e1[sl], eps2=e2[sl])
    torch.cuda.synchronize()
    if rank == 0:
        q.put(torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["sac", "goac", "poac", "ptrain"])
def test_dp_trainer_two_ranks_equals_single_gpu_on_global_batch(kind):
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    tr = _trainer(False, kind)
    for step, (batch, e1, e2) in enumerate(_inputs(world)):
        if kind in ("goac", "ptrain"):
            tr.train_from_torch(_with_counts(batch, step))
        elif kind == "poac":
            tr.train_from_torch(_with_counts(batch, step), eps1=e1, eps2=e2)
        else:
            tr.train_from_torch(batch, eps1=e1, eps2=e2)
    want = torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy()
    assert parity.rel_err(got, want) < 1e-6, parity.rel_err(got, want)


def _ring_run(tr, n_calls, n_steps):
    """n_calls train_from_ring calls of n_steps each on a seeded device replay."""
    from oac_amd import DeviceIndexStream, ReplayBuffer
    from gpu_helpers import Space
    rb = ReplayBuffer(2000, Space(Do), Space(Da), device="cuda:0")
    data = synthetic_transitions(2000, Do, Da, seed=1)
    rb.load_transitions(torch.from_numpy(rb._rows_from(
        data["observations"], data["actions"], data["rewards"], data["next_observations"],
        data["terminals"])).cuda())
    st = DeviceIndexStream(rb, BL, chunk=8, seed=4)
    for _ in range(n_calls):
        st.before_step(n_steps)
        tr.train_from_ring(rb._storage, st.ring, st.slots, BL, n_steps=n_steps)
    torch.cuda.synchronize()
    return torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy()


def _nccl_worker(port, q):
    import faulthandler
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    os.makedirs(os.path.join(os.path.dirname(here), "gpurun_out"), exist_ok=True)
    trace = open(os.path.join(os.path.dirname(here), "gpurun_out", "dp_nccl_worker_stack.txt"), "w")
    faulthandler.dump_traceback_later(90, exit=True, file=trace)   # a hang leaves its stack
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    tr = _trainer(True)
    assert tr.capture
    got = _ring_run(tr, 4, 4)          # call 1 eager, calls 2.. captured (RCCL inside the graph)
    n_graphs = len(tr._graphs)
    dist.destroy_process_group()
    q.put((got, n_graphs))


def test_dp_rccl_graph_capture_single_rank_equals_single_gpu():
    """The captured data-parallel step (phases + RCCL all-reduces in one
    hipGraph, 4 steps per replay) on one rank equals the single-GPU trainer on
    the same device index stream."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_nccl_worker, args=(port, q))
    p.start()
    p.join(timeout=150)
    assert p.exitcode == 0, p.exitcode
    got, n_graphs = q.get()
    assert n_graphs == 1
    want = _ring_run(_trainer(False), 4, 4)
    assert parity.rel_err(got, want) < 1e-6, parity.rel_err(got, want)
