"""Data-parallel path on CPU (gloo, world_size 2): the transport-agnostic
driver oac_amd.dp.dp_step with an oracle-backed executor must reproduce the
single-process step on the concatenated global batch (SURVEY 8e "Parity for
DP").  The GPU executor runs the same driver over RCCL (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fixtures_lib import sac_params, synthetic_transitions
import parity

Do, Da, H, BL, STEPS = 11, 3, [32, 32], 16, 3


class OracleExecutor:
    def __init__(self, orc, batch, e1, e2, world, split=False):
        self.o, self.b, self.e1, self.e2, self.w = orc, batch, e1, e2, world
        self.auto_alpha = orc.auto_alpha
        # the GPU executor's phase-1 split (sac_plan phases 4 / 5): the oracle's
        # phase 1 is one piece, so "1a" (the critics on the fresh actions) is
        # folded into "1b"
        self.split_phase1 = split

    def phase(self, i):
        if i == "1a":
            return
        if i == "1b":
            i = 1
        if i == 0:
            self.o.phase0(self.b, self.e1, self.e2)
        elif i == 1:
            self.o.phase1(self.w)
        elif i == 2:
            self.o.phase2(self.w)
        else:
            self.o.phase3(self.w)

    def alpha_sum(self):
        return self.o.alpha_sum

    def critic_grads(self):
        return self.o.crit_flat

    def policy_grads(self):
        return self.o.pol_flat


def _inputs(world):
    data = synthetic_transitions(500, Do, Da, seed=0)
    rs = np.random.RandomState(5)
    steps = []
    for _ in range(STEPS):
        idx = rs.randint(0, 500, BL * world)
        e1 = rs.standard_normal((BL * world, Da)).astype(np.float32)
        e2 = rs.standard_normal((BL * world, Da)).astype(np.float32)
        steps.append(({k: v[idx] for k, v in data.items()}, e1, e2))
    return steps


def _make(auto_alpha):
    from oracle import sac_oracle as so
    p = sac_params(Do, Da, H, 3, pi_init_w=0.2, q_init_w=0.1)
    return so.SACOracle(p, Do, Da, auto_alpha=auto_alpha, policy_lr=1e-3, qf_lr=1e-3)


def _worker(rank, world, port, auto_alpha, out, overlap=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oac_amd.dp import dp_step
    orc = _make(auto_alpha)
    for batch, e1, e2 in _inputs(world):
        sl = slice(rank * BL, (rank + 1) * BL)
        shard = {k: v[sl] for k, v in batch.items()}
        ex = OracleExecutor(orc, shard, e1[sl], e2[sl], world, split=overlap)

        def ar_async(t):   # the exchange in flight while "1a" runs; join = wait
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
            return work.wait
        dp_step(ex, lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM),
                ar_async if overlap else None)
    if rank == 0:
        flat = torch.cat([t.reshape(-1) for d in (orc.P, orc.Q1, orc.Q2, orc.T1, orc.T2)
                          for t in d.values()] + [orc.log_alpha])
        out.put(flat.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("auto_alpha,overlap", [(True, False), (False, False), (True, True)])
def test_dp_two_ranks_equals_single_process_on_global_batch(auto_alpha, overlap):
    """overlap: the alpha exchange issued asynchronously beside phase "1a"
    and joined before "1b" (dp_step's overlapped schedule)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, auto_alpha, q, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _make(auto_alpha)
    for batch, e1, e2 in _inputs(world):
        ref.step(batch, e1, e2)
    want = torch.cat([t.reshape(-1) for d in (ref.P, ref.Q1, ref.Q2, ref.T1, ref.T2)
                      for t in d.values()] + [ref.log_alpha]).numpy()
    assert parity.rel_err(got, want) < 1e-6
    assert np.max(np.abs(got - want)) < 1e-5


# ---------------------------------------------------------------- g-oac
class GaussOracleExecutor:
    """GaussianOACOracle phases behind the dp_step executor interface (no
    alpha: the phase-0 exchange is skipped, like the GPU executor's)."""
    auto_alpha = False

    def __init__(self, orc, batch, world):
        self.o, self.b, self.w = orc, batch, world

    def phase(self, i):
        if i == 0:
            self.o.phase0(self.b)
        else:
            getattr(self.o, f"phase{i}")(self.w)

    def critic_grads(self):
        return self.o.crit_flat

    def policy_grads(self):
        return self.o.pol_flat


def _goac_make():
    from fixtures_lib import goac_params
    from oracle import sac_oracle as so
    p = goac_params(Do, Da, H, 3, 0.0, 100.0, pi_init_w=0.2, q_init_w=0.1)
    return so.GaussianOACOracle(p, Do, Da, q_min=0.0, q_max=100.0, policy_lr=1e-3, qf_lr=1e-3)


def _goac_inputs(world):
    out = []
    for s, (batch, _, _) in enumerate(_inputs(world)):
        rs = np.random.RandomState(100 + s)
        n = BL * world
        b = dict(batch, counts=(rs.randint(0, 3, (n, 1)) * (rs.uniform(0, 1, (n, 1)) < 0.5)))
        out.append(b)
    return out


def _goac_flat(orc):
    return torch.cat([t.reshape(-1) for d in (orc.P, orc.TP, orc.Q, orc.T)
                      for t in d.values()]).numpy()


def _goac_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oac_amd.dp import dp_step
    orc = _goac_make()
    for batch in _goac_inputs(world):
        sl = slice(rank * BL, (rank + 1) * BL)
        ex = GaussOracleExecutor(orc, {k: v[sl] for k, v in batch.items()}, world)
        dp_step(ex, lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM))
    if rank == 0:
        out.put(_goac_flat(orc))
    dist.barrier()
    dist.destroy_process_group()


def test_goac_dp_two_ranks_equals_single_process_on_global_batch():
    """g-oac (GaussianTrainer) data-parallel step over gloo, counts=True."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_goac_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _goac_make()
    for batch in _goac_inputs(world):
        ref.step(batch)
    want = _goac_flat(ref)
    assert parity.rel_err(got, want) < 1e-6
    assert np.max(np.abs(got - want)) < 1e-5


# ------------------------------------------------- p-oac (particle_trainer.py)
def _ptrain_make():
    from fixtures_lib import ptrain_params
    from oracle import sac_oracle as so
    p = ptrain_params(Do, Da, H, 3, 5, 0.0, 50.0, pi_init_w=0.2, q_init_w=0.1)
    return so.ParticleUBOracle(p, Do, Da, 5, 3, q_min=0.0, q_max=50.0, policy_lr=1e-3,
                               qf_lr=1e-3)


def _ptrain_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oac_amd.dp import dp_step
    orc = _ptrain_make()
    for batch in _goac_inputs(world):
        sl = slice(rank * BL, (rank + 1) * BL)
        ex = GaussOracleExecutor(orc, {k: v[sl] for k, v in batch.items()}, world)
        dp_step(ex, lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM))
    if rank == 0:
        out.put(_goac_flat(orc))
    dist.barrier()
    dist.destroy_process_group()


def test_ptrain_dp_two_ranks_equals_single_process_on_global_batch():
    """p-oac ParticleTrainer data-parallel step over gloo, counts=True (the
    sorted-particle targets and the quantile policy seed are per row; the
    critic / policy gradients are the only exchanges)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_ptrain_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _ptrain_make()
    for batch in _goac_inputs(world):
        ref.step(batch)
    want = _goac_flat(ref)
    assert parity.rel_err(got, want) < 1e-6
    assert np.max(np.abs(got - want)) < 1e-5
