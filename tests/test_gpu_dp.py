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

def _spawn(target, args_of, world=1, n_get=1, timeout=240):
    """Start ``world`` spawned workers target(*args_of(rank, port, q)), read
    ``n_get`` results BEFORE joining (a worker blocks in q.put until its
    message -- a state larger than the pipe's buffer -- is read), each read
    bounded by ``timeout`` (a worker that dies without putting fails the test
    instead of hanging it), then join and check every exit code."""
    import queue as _queue
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=args_of(r, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = [q.get(timeout=timeout) for _ in range(n_get)]
    except _queue.Empty:
        for p in procs:
            p.join(timeout=5)
        raise AssertionError(("no result from a worker", [p.exitcode for p in procs]))
    for p in procs:
        p.join(timeout=timeout)
        assert p.exitcode == 0, p.exitcode
    return got


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


def _trainer(dp, kind="sac", transport=None):
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
    kw = {"rccl1": dict(force_collectives=True),
          # the split schedule of the world > 1 RCCL step (phase "1a", the
          # alpha exchange, phase "1b" = library phases 4 / 5)
          "rccl1_overlap": dict(force_collectives=True, force_overlap=True),
          "overlap": dict(force_overlap=True)}.get(dp, {})
    if dp and transport:
        kw["transport"] = transport
    return cls(pp, qp, action_space=Space(Da), discount=0.99, reward_scale=1.0, policy_lr=1e-3,
               qf_lr=1e-3, soft_target_tau=5e-3, use_automatic_entropy_tuning=True, **kw)


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
    tr = _trainer("overlap" if kind == "sac_overlap" else True, kind)
    assert tr._overlap == (kind == "sac_overlap")
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


@pytest.mark.parametrize("kind", ["sac", "sac_overlap", "goac", "poac", "ptrain"])
def test_dp_trainer_two_ranks_equals_single_gpu_on_global_batch(kind):
    """sac_overlap: the split schedule (phases 4 / 5 of sac_plan.hip with the
    alpha all-reduce between them, synchronous over gloo) -- the library code
    only the world > 1 RCCL step runs otherwise."""
    world = 2
    got, = _spawn(_worker, lambda r, port, q: (r, world, port, q, kind), world)
    tr = _trainer(False, "sac" if kind == "sac_overlap" else kind)
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


def _nccl_worker(port, q, teardown="close", overlap=False, transport="torch"):
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
    tr = _trainer("rccl1_overlap" if overlap else "rccl1", transport=transport)
    assert tr._overlap == overlap and tr.transport == transport
    got = _ring_run(tr, 4, 4)          # torch: call 1 eager, calls 2.. captured (RCCL inside the graph)
    if transport == "torch":
        n = len(tr._graphs)
    else:   # the library's own communicator, exchanges issued between its launches
        from oac_amd import _lib
        n = _lib.lib().oac_sac_trace(tr._last_plan.handle, 1)
    q.put((got, n))
    if teardown == "close":
        # the trainer's own teardown, then the process group: destroying the
        # group under live graphs (they hold RCCL kernels) aborted the process
        tr.close()
        assert not tr._graphs and tr._rccl is None
        dist.destroy_process_group()
    # "atexit": neither -- the trainer's atexit hook releases the graphs


@pytest.mark.parametrize("teardown,overlap,transport",
                         [("close", False, "torch"), ("atexit", False, "torch"), ("close", True, "torch"),
                          ("close", False, "library"), ("atexit", True, "library")])
def test_dp_rccl_graph_capture_single_rank_equals_single_gpu(teardown, overlap, transport):
    """The captured data-parallel step (phases + RCCL all-reduces in one
    hipGraph, 4 steps per replay) on one rank equals the single-GPU trainer on
    the same device index stream, and the process exits cleanly through the
    trainer's teardown (explicit close(), or its atexit hook).  overlap: the
    world > 1 schedule -- phase "1a", the alpha all-reduce on a forked side
    stream captured into the graph as a fork / join, phase "1b".
    transport="library": no graph -- the library issues the three RCCL
    all-reduces itself on its own communicator between its launches (the
    split schedule on its side stream), checked through the plan's trace."""
    (got, n), = _spawn(_nccl_worker, lambda r, port, q: (port, q, teardown, overlap, transport))
    if transport == "torch":
        assert n == 1   # one captured graph
    else:
        from oac_amd._lib import TRACE
        assert n & TRACE["exchange"] and not n & TRACE["fused"], n
        assert bool(n & TRACE["split_phase1"]) == overlap, n
    want = _ring_run(_trainer(False), 4, 4)
    assert parity.rel_err(got, want) < 1e-6, parity.rel_err(got, want)


# ---------------------------------------------------------------- configs[3]
# BASELINE configs[3] at its per-rank scale: Humanoid dims, 2x256 MLPs, per-rank
# batch 4096, two ranks (gloo on one GPU).  The data-parallel HIP step must
# equal the single-GPU step on the concatenated 8,192-row batch, and both the
# CPU oracle on that batch (SURVEY 8e "Parity for DP").
HD, HA, HH, HB = 376, 17, 256, 4096


def _h_inputs(world, steps=2):
    data = synthetic_transitions(3 * HB * world, HD, HA, seed=0)
    rs = np.random.RandomState(9)
    out = []
    for _ in range(steps):
        idx = rs.randint(0, len(data["rewards"]), HB * world)
        e1 = rs.standard_normal((HB * world, HA)).astype(np.float32)
        e2 = rs.standard_normal((HB * world, HA)).astype(np.float32)
        out.append(({k: v[idx] for k, v in data.items()}, e1, e2))
    return out


def _h_trainer(dp, **kw):
    from gpu_helpers import producers, Space
    from oac_amd import SACTrainer
    from oac_amd.dp import DataParallelSACTrainer
    pp, qp = producers(sac_params(HD, HA, [HH, HH], 4, pi_init_w=1e-3, q_init_w=3e-3))
    cls = DataParallelSACTrainer if dp else SACTrainer
    return cls(pp, qp, action_space=Space(HA), discount=0.99, reward_scale=1.0, policy_lr=3e-4,
               qf_lr=3e-4, soft_target_tau=5e-3, use_automatic_entropy_tuning=True, **kw)


def _flat_state(tr):
    return torch.cat([tr.params, tr.targets, tr.alpha_state[:4]]).cpu().numpy()


def _h_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = _h_trainer(True)
    grads0 = None
    for step, (batch, e1, e2) in enumerate(_h_inputs(world)):
        sl = slice(rank * HB, (rank + 1) * HB)
        tr.train_from_torch({k: v[sl] for k, v in batch.items()}, eps1=e1[sl], eps2=e2[sl])
        if step == 0:   # the all-reduced SUM of the ranks' gradients
            grads0 = (tr.grads / world).cpu().numpy()
    torch.cuda.synchronize()
    if rank == 0:
        q.put((grads0, _flat_state(tr)))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_humanoid_b4096_two_ranks_equals_single_gpu_and_oracle():
    from gpu_helpers import module_tensors
    from oracle import sac_oracle as so
    world = 2
    (dp_grads0, dp_state), = _spawn(_h_worker, lambda r, port, q: (r, world, port, q), world)
    inputs = _h_inputs(world)
    tr = _h_trainer(False)
    single_grads0 = None
    for step, (batch, e1, e2) in enumerate(inputs):
        tr.train_from_torch(batch, eps1=e1, eps2=e2)
        if step == 0:
            single_grads0 = tr.grads.clone()
    torch.cuda.synchronize()
    # DP == single GPU on the global batch
    assert parity.rel_err(dp_grads0, single_grads0.cpu().numpy()) < 1e-5
    assert parity.rel_err(dp_state, _flat_state(tr)) < 1e-5
    # both == the CPU oracle on the global batch, per tensor (step 0 gradients)
    orc = so.SACOracle(sac_params(HD, HA, [HH, HH], 4, pi_init_w=1e-3, q_init_w=3e-3), HD, HA,
                       policy_lr=3e-4, qf_lr=3e-4, tau=5e-3)
    batch, e1, e2 = inputs[0]
    out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
    dp_view = torch.from_numpy(dp_grads0).to(tr.grads.device)
    # ReLU-boundary entries of the critics' hidden layers (parity.relu_boundary_units):
    # the only rows a correct fp32 step may disagree on at this batch size
    prm = sac_params(HD, HA, [HH, HH], 4, pi_init_w=1e-3, q_init_w=3e-3)
    x0 = np.concatenate([batch["observations"], batch["actions"]], 1)
    allowed = {}
    for grp in ("qf1", "qf2"):
        q = prm[grp]
        u0, pre0 = parity.relu_boundary_units(x0, q["fc0.weight"], q["fc0.bias"])
        u1, _ = parity.relu_boundary_units(np.maximum(pre0, 0), q["fc1.weight"], q["fc1.bias"])
        allowed[grp] = {"fc0.weight": u0, "fc0.bias": u0, "fc1.weight": u1, "fc1.bias": u1}
    left_out = {}
    for grp, mod in (("policy", tr.policy), ("qf1", tr.qf1), ("qf2", tr.qf2)):
        got_single = module_tensors(tr, mod, single_grads0)
        got_dp = module_tensors(tr, mod, dp_view)
        for name, ref in out["grads"][grp].items():
            ref = ref.numpy()
            rows = allowed.get(grp, {}).get(name, [])
            for tag, got in (("single", got_single), ("dp", got_dp)):
                e, bad = parity.rel_err_rows(got[name].cpu().numpy(), ref, rows)
                assert e < 1e-5, (tag, grp, name, e, rows)
                if bad:
                    left_out[(tag, grp, name)] = bad
    print("ReLU-boundary rows left out:", left_out)


def _dropin_worker(rank, world, port, q, dropin):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oac_amd import ReplayBuffer
    from gpu_helpers import Space
    tr = _trainer(True)
    tr._no_dropin = not dropin   # False: the device-index path (indices uploaded, no ring)
    rb = ReplayBuffer(500, Space(Do), Space(Da), device="cuda:0")
    d = synthetic_transitions(500, Do, Da, seed=rank)
    rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                       rewards=d["rewards"], next_observations=d["next_observations"],
                       terminals=d["terminals"])])
    np.random.seed(1 + rank)
    for _ in range(140):        # past the 128-slot staging ring
        b = rb.random_batch(BL)
        b["buffer"] = rb
        tr.train(b)
    torch.cuda.synchronize()
    if rank == 0:
        q.put(torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def _dropin_loop(tr, seed=1, steps=140):
    from oac_amd import ReplayBuffer
    from gpu_helpers import Space
    rb = ReplayBuffer(500, Space(Do), Space(Da), device="cuda:0")
    d = synthetic_transitions(500, Do, Da, seed=0)
    rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                       rewards=d["rewards"], next_observations=d["next_observations"],
                       terminals=d["terminals"])])
    np.random.seed(seed)
    for _ in range(steps):        # past the 128-slot staging ring
        b = rb.random_batch(BL)
        b["buffer"] = rb
        tr.train(b)
    torch.cuda.synchronize()
    return torch.cat([tr.params, tr.targets, tr.alpha_state[:3]]).cpu().numpy()


def _nccl_dropin_worker(port, q, overlap=False, transport="torch"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    tr = _trainer("rccl1_overlap" if overlap else "rccl1", transport=transport)
    assert tr._overlap == overlap
    got = _dropin_loop(tr)
    q.put((got, len(tr._attached) if transport == "torch" else 1))
    tr.close()
    assert not tr._attached
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap,transport", [(False, "torch"), (True, "torch"), (False, "library"),
                                               (True, "library")])
def test_dp_rccl_dropin_step_graph_equals_single_gpu(overlap, transport):
    """The drop-in loop on the data-parallel trainer over RCCL (one rank): from
    the third call on, the captured step (phases + RCCL all-reduces) is
    attached to the handle and each train() is one library call (staging +
    graph launch); 140 steps across the staging ring's wrap equal the
    single-process drop-in step."""
    (got, n_attached), = _spawn(_nccl_dropin_worker, lambda r, port, q: (port, q, overlap, transport))
    assert n_attached == 1
    want = _dropin_loop(_trainer(False))
    assert parity.rel_err(got, want) < 1e-6, parity.rel_err(got, want)


def test_dp_dropin_loop_equals_device_index_path():
    """rl_algorithm.py:160-167 on every rank (own replay shard, own numpy
    seed): the staged host-index path equals the device-index path."""
    world = 2
    got = {}
    for dropin in (True, False):
        got[dropin], = _spawn(_dropin_worker, lambda r, port, q: (r, world, port, q, dropin), world)
    assert np.array_equal(got[True], got[False])


# ------------------------------------------- the 8-GPU step's code at BASELINE dims
# bench.py --gpus 8 runs the drop-in loop on DataParallelSACTrainer over RCCL
# with the split schedule on (dp.py: _overlap at world > 1): at B=4096 per rank
# phase 0 gathers directly (direct_big), phase 4 carries the batch copy, the
# targets kernel the width-1 heads' partials (qdot) and the last layers' dW
# slabs (wl_in_targets).  These tests run exactly that code at Humanoid dims.
NR = 20000
BIG_BRANCHES = ("direct_big", "batch_copy", "qdot", "wl_targets", "split_phase1", "exchange")


def _h_replay(seed):
    from oac_amd import ReplayBuffer
    from gpu_helpers import Space
    rb = ReplayBuffer(NR, Space(HD), Space(HA), device="cuda:0")
    d = synthetic_transitions(NR, HD, HA, seed=seed)
    rb.add_paths([dict(observations=d["observations"], actions=d["actions"],
                       rewards=d["rewards"], next_observations=d["next_observations"],
                       terminals=d["terminals"])])
    return rb, d


def _h_dropin_worker(rank, world, port, q, steps, overlap):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oac_amd import _lib
    tr = _h_trainer(True, force_overlap=overlap, seed=rank)
    assert tr.transport == "library" and tr._overlap == overlap
    rb, _ = _h_replay(10 + rank)                              # this rank's shard
    np.random.seed(1 + rank)                                  # this rank's index stream
    recs, grads0 = [], None
    for step in range(steps):
        b = rb.random_batch(HB)
        b["buffer"] = rb
        tr.train(b)                                           # rl_algorithm.py:160-167
        torch.cuda.synchronize()
        v = tr._last_plan.views
        recs.append((np.array(b.host_indices), v["eps1"].cpu().numpy(), v["eps2"].cpu().numpy()))
        if step == 0:
            grads0 = (tr.grads / world).cpu().numpy()
    trace = _lib.lib().oac_sac_trace(tr._last_plan.handle, 1)
    q.put((rank, recs, grads0 if rank == 0 else None, _flat_state(tr) if rank == 0 else None, trace))
    dist.barrier()
    tr.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
def test_dp_humanoid_b4096_two_ranks_split_schedule_dropin_equals_single_gpu_and_oracle(overlap):
    """configs[3] per rank (Humanoid, B=4096, own replay shard and index
    stream per rank, Philox eps), two ranks over gloo, through the drop-in
    call -- the exact code path of the 8-GPU run: phases 0, [alpha exchange],
    1, [critic grads], 2, [policy grads], 3 issued by the library, with the
    large-batch branches (trace); overlap: the split schedule (phases 4 / 5
    with the alpha exchange on the plan's side stream, OAC_DP_OVERLAP).  Against the single-GPU step on the
    concatenated 8,192 rows with the ranks' own eps, and the oracle (step 0)."""
    from gpu_helpers import module_tensors
    from oac_amd._lib import TRACE
    from oracle import sac_oracle as so
    world, steps = 2, 2
    got = dict((m[0], m[1:]) for m in _spawn(
        _h_dropin_worker, lambda r, port, q: (r, world, port, q, steps, overlap), world, n_get=2))
    dp_grads0, dp_state = got[0][1], got[0][2]
    for r in range(world):
        tr_bits = got[r][3]
        missing = [b for b in BIG_BRANCHES if b != "split_phase1" and not tr_bits & TRACE[b]]
        assert not missing, (r, missing, tr_bits)
        assert bool(tr_bits & TRACE["split_phase1"]) == overlap, tr_bits
    shards = [synthetic_transitions(NR, HD, HA, seed=10 + r) for r in range(world)]
    inputs = []
    for step in range(steps):
        parts = [({k: v[got[r][0][step][0]] for k, v in shards[r].items()}, got[r][0][step][1],
                  got[r][0][step][2]) for r in range(world)]
        batch = {k: np.concatenate([p[0][k] for p in parts]) for k in parts[0][0]}
        inputs.append((batch, np.concatenate([p[1] for p in parts]),
                       np.concatenate([p[2] for p in parts])))
    tr = _h_trainer(False)
    single0 = None
    for step, (batch, e1, e2) in enumerate(inputs):
        tr.train_from_torch(batch, eps1=e1, eps2=e2)
        if step == 0:
            single0 = tr.grads.clone()
            # the layer-1 masks the step's critic backward used (8,192 rows)
            h2g = {g: tr._last_plan.views["h2q" + g[-1]].cpu().numpy() for g in ("qf1", "qf2")}
    torch.cuda.synchronize()
    e_g, e_s = parity.rel_err(dp_grads0, single0.cpu().numpy()), parity.rel_err(dp_state, _flat_state(tr))
    print("dp vs single: grads0 %.2e, state after %d steps %.2e" % (e_g, steps, e_s))
    assert e_g < 1e-5 and e_s < 1e-5
    # step 0 against the oracle on the global batch, per tensor (ReLU-boundary
    # rows of the critics' hidden layers aside, as in the test above; a
    # critic's fc0 against the oracle corrected by exactly the layer-1 mask
    # flips the GPU's saved activations show, each within 3e-5 rms of 0:
    # test_gpu_teacher._flip_adjusted)
    from test_gpu_teacher import _flip_adjusted
    prm = sac_params(HD, HA, [HH, HH], 4, pi_init_w=1e-3, q_init_w=3e-3)
    orc = so.SACOracle(prm, HD, HA, policy_lr=3e-4, qf_lr=3e-4, tau=5e-3)
    batch, e1, e2 = inputs[0]
    out = orc.step(so.NumpyReplay.to_torch(batch), e1, e2)
    Bg = len(batch["rewards"])
    flipped = {}
    for grp, c, opt in (("qf1", "c1", orc.opt_q1), ("qf2", "c2", orc.opt_q2)):
        dq = 2.0 * (orc.S[c]["q"] - orc.S["y"]) / Bg
        adj, fl = _flip_adjusted(out["grads"][grp], orc.S[c], dq, prm[grp], opt, 3e-4, h2g[grp])
        flipped[grp] = fl
        for pn in ("fc0.weight", "fc0.bias"):
            out["grads"][grp][pn] = torch.from_numpy(adj[pn][0])
    print("layer-1 mask flips (sample, unit):", flipped)
    x0 = np.concatenate([batch["observations"], batch["actions"]], 1)
    allowed = {}
    for grp in ("qf1", "qf2"):
        qq = prm[grp]
        u0, pre0 = parity.relu_boundary_units(x0, qq["fc0.weight"], qq["fc0.bias"])
        u1, _ = parity.relu_boundary_units(np.maximum(pre0, 0), qq["fc1.weight"], qq["fc1.bias"])
        allowed[grp] = {"fc0.weight": u0, "fc0.bias": u0, "fc1.weight": u1, "fc1.bias": u1}
    dp_view = torch.from_numpy(dp_grads0).to(tr.grads.device)
    for grp, mod in (("policy", tr.policy), ("qf1", tr.qf1), ("qf2", tr.qf2)):
        got_dp = module_tensors(tr, mod, dp_view)
        for name, ref in out["grads"][grp].items():
            e, _ = parity.rel_err_rows(got_dp[name].cpu().numpy(), ref.numpy(),
                                       allowed.get(grp, {}).get(name, []))
            assert e < 1e-5, (grp, name, e)


def _nccl_h_worker(port, q, B, steps, overlap):
    import faulthandler
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    os.makedirs(os.path.join(os.path.dirname(here), "gpurun_out"), exist_ok=True)
    trace = open(os.path.join(os.path.dirname(here), "gpurun_out", "dp_nccl_h_worker_stack.txt"), "w")
    faulthandler.dump_traceback_later(100, exit=True, file=trace)
    for p in (here, os.path.join(os.path.dirname(here), "oac-explore_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from oac_amd import _lib
    tr = _h_trainer(True, force_collectives=True, force_overlap=overlap)
    rb, _ = _h_replay(7)
    np.random.seed(3)
    for _ in range(steps):
        b = rb.random_batch(B)
        b["buffer"] = rb
        tr.train(b)
    torch.cuda.synchronize()
    bits = _lib.lib().oac_sac_trace(tr._last_plan.handle, 1)
    q.put((_flat_state(tr), bits))
    tr.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("B", [256, 4096])
def test_dp_rccl_humanoid_split_schedule_dropin_equals_single_gpu(B, overlap):
    """The 8-GPU step's code over RCCL at one rank, Humanoid dims at the
    headline batch (256) and configs[3]'s (4096): the library's own
    communicator, the three all-reduces issued between its launches --
    in line (overlap False: the world > 1 default, dp.py) or with the alpha
    exchange on the side stream beside phase 4 (overlap True) -- through the
    drop-in call, against the single-process drop-in step on the same
    replay, index stream and Philox eps."""
    from oac_amd._lib import TRACE
    steps = 24
    (got, bits), = _spawn(_nccl_h_worker, lambda r, port, q: (port, q, B, steps, overlap))
    want_bits = ("direct", "head_dh2") if B == 256 else BIG_BRANCHES
    missing = [b for b in want_bits + ("exchange",) if b != "split_phase1" and not bits & TRACE[b]]
    assert not missing and not bits & TRACE["fused"], (missing, bits)
    assert bool(bits & TRACE["split_phase1"]) == overlap, bits
    tr = _h_trainer(False)
    rb, _ = _h_replay(7)
    np.random.seed(3)
    for _ in range(steps):
        b = rb.random_batch(B)
        b["buffer"] = rb
        tr.train(b)
    torch.cuda.synchronize()
    e = parity.rel_err(got, _flat_state(tr))
    print("B=%d DP (RCCL, split schedule) vs single-process: %.2e" % (B, e))
    assert e < 1e-5
