"""Data-parallel OAC/SAC step over RCCL (BASELINE configs[3]).

One process per GPU, each with its own replay shard and its own index
stream; parameters, Adam state and targets are replicated.  The reference has
no distributed path (it runs one independent seed per GPU, main.py:575-578);
this is the DP scheme the build adds.  Per step there are exactly three
exchanges, at the points where the single-GPU step needs a whole-batch
quantity, in the torch-1.4 order of trainer.py:139-210:

  phase 0   forward, policy sample, local sum(logp + H) as
            per-16-row partials (the head launch)              -> all-reduce SUM (B/16 floats)
  phase 1   alpha update (global sum), TD target, critic grads -> all-reduce SUM (1.34 MB)
  phase 2   critic Adam (grads / world) + Polyak, policy grad
            through the post-step critics                       -> all-reduce SUM (0.68 MB)
  phase 3   policy Adam (grads / world), step advance

With equal per-rank batches and mean-reduced losses, the averaged gradients
are the gradients of the concatenated global batch, so a DP step equals the
single-process step on the union of the ranks' batches (tests/test_dp.py
checks this with the CPU oracle over gloo).

The exchanges are issued by liboac_amd itself, between its own launches
(``oac_sac_set_allreduce``, sac_plan.hip ``run_step_dp``): over RCCL through
the library's own communicator (``oac_rccl_*``, bootstrapped from the process
group; the nccl backend) or, over gloo, through a host callback into
torch.distributed (tests).  A step is then one library call of direct
launches and stream-ordered all-reduces, like the single-process step.

``dp_step`` is the transport-agnostic Python driver of the same sequence: the
CPU tests run it with an oracle-backed executor over gloo, and
``OAC_DP_TRANSPORT=torch`` (or ``transport="torch"``) keeps the round-1..4
GPU path -- the library's phases driven from Python with torch's
all-reduces, RCCL steps captured into a torch graph -- for A/B runs.
"""
import atexit
import ctypes
import os
import weakref

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import check
from .gaussian_trainer import GaussianTrainer
from .particle_trainer import ParticleTrainer
from .particle_trainer_oac import ParticleTrainer as ParticleTrainerOAC
from .trainer import SACTrainer


def dp_step(ex, all_reduce, all_reduce_async=None):
    """Drive one data-parallel step.  ``ex`` exposes phase(i) and the views
    alpha_sum() / critic_grads() / policy_grads(); ``all_reduce(t)`` sums a
    tensor over ranks in place (the executor's Adam divides by world size).
    With ``all_reduce_async(t) -> join`` and an executor that splits phase 1
    (``ex.split_phase1``: "1a" = the critics on the fresh actions, which need
    no alpha, "1b" = the rest), the alpha exchange runs beside "1a"."""
    ex.phase(0)
    if ex.auto_alpha and all_reduce_async is not None and getattr(ex, "split_phase1", False):
        join = all_reduce_async(ex.alpha_sum())
        ex.phase("1a")
        join()
        ex.phase("1b")
    else:
        if ex.auto_alpha:
            all_reduce(ex.alpha_sum())
        ex.phase(1)
    all_reduce(ex.critic_grads())
    ex.phase(2)
    all_reduce(ex.policy_grads())
    ex.phase(3)


class _GpuExecutor:
    def __init__(self, trainer, plan, flags, stream):
        self.t, self.plan, self.flags, self.stream = trainer, plan, flags, stream
        self.auto_alpha = trainer.use_automatic_entropy_tuning
        self.split_phase1 = trainer._kind == _lib.OAC_KIND_SAC   # phases 4 / 5 (sac_plan.hip)
        lay = trainer.layout
        self._crit = trainer.grads[lay.q1_base:lay.q1_base + lay.n_critics * lay.q_size]
        self._pol = trainer.grads[:lay.q1_base]   # policy Adam group

    _SPLIT = {"1a": 4, "1b": 5}

    def phase(self, i):
        # every phase sees the step flags: phase 0 gathers / draws, phase 1
        # reads OAC_STEP_COUNTS (particle / gaussian targets)
        check(_lib.lib().oac_sac_step_phase(self.plan.handle, self._SPLIT.get(i, i), self.flags,
                                            _lib.stream_ptr(self.stream)))

    def alpha_sum(self):
        # the head launch's per-16-row partials of sum(logp + target_entropy)
        # (OAC_WS_LOGP_PART); the targets kernel sums the all-reduced vector
        return self.plan.views["logp_part"].view(-1)

    def critic_grads(self):
        return self._crit

    def policy_grads(self):
        return self._pol


def _librccl_path():
    """The librccl.so torch's process group uses (so the library's
    communicator and torch's share one RCCL instance), else ROCm's."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "/opt/rocm/lib/librccl.so"


def _close_at_exit(ref):
    tr = ref()
    if tr is not None and dist.is_initialized():
        try:
            tr.close()
        except Exception:   # interpreter exit: the device may already be gone
            pass


class _DataParallel:
    """Mixin: the trainer's step sharded over the ranks of a process group
    (NCCL backend = RCCL on ROCm).  Every rank builds the trainer the same way;
    rank 0's initial state is broadcast.

    With RCCL, the ring fast path (``train_from_ring``) captures whole steps --
    the four phase launch sequences AND the three all-reduces -- into one
    hipGraph per (plan, n_steps) after one eager call, so a step costs one
    graph replay instead of ~20 host-issued launches and collectives
    (``capture=False`` keeps every step eager)."""

    def __init__(self, *args, process_group=None, capture=None, force_collectives=False,
                 force_overlap=False, transport=None, **kwargs):
        if not dist.is_initialized():
            raise RuntimeError("DataParallelSACTrainer needs torch.distributed initialised")
        self.pg = process_group
        # "library": liboac_amd issues the exchanges itself (RCCL communicator
        # of its own, or a host callback over gloo); "torch": Python drives the
        # phases with torch's all-reduces (the round-1..4 path, A/B runs)
        self.transport = transport or os.environ.get("OAC_DP_TRANSPORT", "library")
        if self.transport not in ("library", "torch"):
            raise ValueError(f"transport {self.transport!r}: 'library' or 'torch'")
        self._force = force_collectives
        self._rccl = None          # the library's communicator (oac_rccl*), created on first use
        self._ar = None            # (fn, ctx) of the attached hook
        self._ar_err = None
        self.world = dist.get_world_size(process_group)
        # a sum over one rank is the identity: at world size 1 the exchanges
        # are skipped (force_collectives=True issues them anyway: what the
        # collective library's captured calls cost, for measurement)
        self._collectives = self.world > 1 or force_collectives
        self.capture = (dist.get_backend(process_group) == "nccl") if capture is None else capture
        # the alpha exchange beside the fresh-action critic forward (RCCL only:
        # with gloo the collective is a host call and there is nothing to
        # overlap; at one rank the all-reduce has no link latency to hide and
        # the fork / join alone cost ~3.7 us per step).  force_overlap=True
        # runs the split schedule anyway -- phase "1a", the alpha exchange,
        # phase "1b" (library phases 4 / 5) -- so the code the world > 1 RCCL
        # step executes can be tested at world size 1 (RCCL: the forked-stream
        # all-reduce captured into the step graph) and over gloo (a
        # synchronous all-reduce between the two halves)
        self._nccl = dist.get_backend(process_group) == "nccl"
        if self.transport == "library":
            # the library's fork / join of the overlapped alpha exchange (an
            # event record + a cross-stream wait each way, direct launches)
            # measured ~24 us per step at one rank over RCCL (7,459 -> 6,321
            # steps/s with the exchanges forced): more than a 16-float
            # all-reduce's link latency, so the exchange stays in line unless
            # asked for (OAC_DP_OVERLAP=1)
            self._overlap = force_overlap or os.environ.get("OAC_DP_OVERLAP") == "1"
        else:
            self._overlap = force_overlap or (self._nccl and self.world > 1
                                              and os.environ.get("OAC_DP_OVERLAP", "1") != "0")
        self._graphs, self._eager_seen = {}, set()
        self._attached = {}   # plan handles a captured step graph is attached to
        self._closed = False
        super().__init__(*args, **kwargs)
        # make sure every rank starts from rank 0's state
        with torch.no_grad():
            for t in (self.params, self.targets, self.alpha_state):
                dist.broadcast(t, src=0, group=process_group)
        # the captured step graphs hold RCCL kernels of the communicator:
        # destroying the process group under live graphs aborts the process,
        # so a trainer nobody closed releases them at interpreter exit (atexit
        # runs last-registered first: before a process-group teardown that
        # was registered earlier)
        atexit.register(_close_at_exit, weakref.ref(self))

    def release_graphs(self):
        """Drop the captured step graphs (they hold RCCL kernels of this
        process group's communicator)."""
        if not self._graphs and not self._eager_seen:
            return
        torch.cuda.synchronize(self.device)
        for h in self._attached.values():   # the handles launch the step graphs: detach first
            check(_lib.lib().oac_sac_set_step_graph(h, None, 0))
        self._attached.clear()
        self._graphs.clear()
        self._eager_seen.clear()
        torch.cuda.synchronize(self.device)

    def close(self):
        """The data-parallel trainer's teardown: finish the queued steps,
        release the captured graphs and the library's communicator, so the
        caller may then destroy the process group
        (``dist.destroy_process_group()``).  Idempotent; a step after close()
        re-captures / re-creates the communicator (collectively)."""
        if self._closed:
            return
        self._closed = True
        self.release_graphs()
        self._side = None
        if self._ar is not None:
            torch.cuda.synchronize(self.device)
            for p in self._plans.values():
                if getattr(p, "hooked", False):
                    check(_lib.lib().oac_sac_set_allreduce(p.handle, None, None, 0))
                    p.hooked = False
            if self._rccl is not None:
                check(_lib.lib().oac_rccl_destroy(self._rccl))
                self._rccl = None
            self._ar = None

    # ---------------------------------------------------- library transport
    def _hook(self):
        """(fn, ctx) of the all-reduce hook the plans carry: the library's RCCL
        communicator (nccl backend; created collectively on first use, its
        unique id broadcast from the group's rank 0) or a host callback into
        torch.distributed (gloo)."""
        if self._ar is not None:
            return self._ar
        L = _lib.lib()
        if self._nccl:
            path = _librccl_path().encode()
            uid = (ctypes.c_char * 128)()
            if dist.get_rank(self.pg) == 0:
                check(L.oac_rccl_unique_id(path, uid))
            obj = [bytes(uid)]
            src = 0 if self.pg is None else dist.get_global_rank(self.pg, 0)
            dist.broadcast_object_list(obj, src=src, group=self.pg, device=self.device)
            ctypes.memmove(uid, obj[0], 128)
            h = ctypes.c_void_p()
            check(L.oac_rccl_create(path, uid, dist.get_rank(self.pg), self.world, ctypes.byref(h)))
            self._rccl = h
            self._ar = (ctypes.cast(L.oac_rccl_allreduce, ctypes.c_void_p), h)
        else:
            self._ar_cb = _lib.ALLREDUCE_FN(self._host_allreduce)
            self._ar = (ctypes.cast(self._ar_cb, ctypes.c_void_p), None)
        self._closed = False
        return self._ar

    def _host_allreduce(self, ctx, buf, n, stream):
        """The hook over a host transport (gloo): the stream's work so far,
        a host all-reduce, the sum copied back before the library continues."""
        try:
            t = self._view_of(buf, n)
            s = (torch.cuda.ExternalStream(stream, device=self.device) if stream
                 else torch.cuda.default_stream(self.device))
            s.synchronize()
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.pg)
            with torch.cuda.stream(s):
                t.copy_(h)
            s.synchronize()
            return 0
        except BaseException as e:   # (a ctypes callback cannot raise through C)
            self._ar_err = e
            return 1

    def _view_of(self, addr, n):
        """The tensor view of the hook's buffer: the grads arena or a plan's workspace."""
        for t in [self.grads] + [p.ws for p in self._plans.values()]:
            b = t.data_ptr()
            if b <= addr and addr + 4 * n <= b + 4 * t.numel():
                o = (addr - b) // 4
                return t[o:o + n]
        raise RuntimeError("all-reduce hook: buffer outside the trainer's arenas")

    def _plan(self, B, *args, **kwargs):
        p = super()._plan(B, *args, **kwargs)
        if self.transport == "library" and not getattr(p, "hooked", False):
            fn, ctx = self._hook()
            flags = ((_lib.OAC_DP_FORCE if self._force else 0)
                     | (_lib.OAC_DP_OVERLAP if self._overlap else 0))
            check(_lib.lib().oac_sac_set_allreduce(p.handle, fn, ctx, flags))
            p.hooked = True
        return p

    def _lib_call(self, fn, *args, **kwargs):
        self._ar_err = None
        try:
            return fn(*args, **kwargs)
        except RuntimeError:
            if self._ar_err is not None:
                raise self._ar_err
            raise

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def _make_cfg(self, batch):
        c = super()._make_cfg(batch)
        c.world_size = self.world
        return c

    def _all_reduce(self, t):
        if self._collectives:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg)

    def _all_reduce_async(self, t):
        """The all-reduce on a side stream forked from the current one; the
        returned join makes the current stream wait for it (captured into the
        step graph as a fork / join, so the exchange overlaps the work issued
        between the fork and the join)."""
        if not self._nccl:   # gloo: a host-side collective, nothing runs beside it
            self._all_reduce(t)
            return lambda: None
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        side = self._side
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self._all_reduce(t)
        return lambda: cur.wait_stream(side)

    def _steps(self, plan, f, n_steps, stream):
        ex = _GpuExecutor(self, plan, f, stream)
        overlap = self._all_reduce_async if self._overlap else None
        for _ in range(n_steps):
            dp_step(ex, self._all_reduce, overlap)

    def _train_host_indices(self, dbatch):
        if self.transport == "library":   # one library call: staging + the DP step
            return self._lib_call(super()._train_host_indices, dbatch)
        return self._train_host_indices_torch(dbatch)

    def _train_host_indices_torch(self, dbatch):
        """The drop-in call (random_batch + train per step) at world > 1: this
        rank's host-drawn indices are staged into the plan's ring, then the
        one-step data-parallel graph (phases + the three all-reduces) runs.
        The first call runs eager, the second captures; from then on the
        captured graph is attached to the handle and a call is one library
        call (staging + graph launch on torch's current stream), as in the
        single-process step -- through torch's replay and the stream hop the
        Python-side call cost ~40 us per step (B=256 at one rank: 7,294 ->
        10,183 steps/s against 10,488 single-process)."""
        plan = self._dropin_plan(dbatch)
        if self._bc_mirror is None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self._bc_mirror = int(self.step_state[1].item())
        idx = dbatch.host_indices
        if idx.dtype != np.int64 or not idx.flags.c_contiguous:
            idx = np.ascontiguousarray(idx, dtype=np.int64)
        bc = self._bc_mirror
        step_flags = _lib.OAC_STEP_GATHER | _lib.OAC_STEP_DEVICE_EPS   # what _run captures
        key = (id(plan), step_flags, 1)
        if self.capture and key in self._graphs and not self._closed:
            # the captured step attached to the handle: staging + one graph
            # launch on torch's current stream in one library call, as the
            # single-process drop-in step (no stream hop, no replay prologue)
            if plan.handle.value not in self._attached:
                check(_lib.lib().oac_sac_set_step_graph(
                    plan.handle, ctypes.c_void_p(self._graphs[key].raw_cuda_graph_exec()),
                    step_flags))
                self._attached[plan.handle.value] = plan.handle
            check(_lib.lib().oac_sac_step_host_idx(
                plan.handle, ctypes.c_void_p(idx.ctypes.data), bc, step_flags,
                _lib.stream_ptr(torch.cuda.current_stream(self.device))))
            self._bc_mirror = bc + 1
            self._last_plan = plan
            if self._need_to_update_eval_statistics:
                self._need_to_update_eval_statistics = False
                self._fill_eval_statistics(plan)
            self._n_train_steps_total += 1
            return

        def stage(sp):
            check(_lib.lib().oac_sac_stage_host_idx(plan.handle, ctypes.c_void_p(idx.ctypes.data),
                                                    bc, sp))
        self._run(plan, _lib.OAC_STEP_GATHER, n_steps=1, pre=stage)
        self._bc_mirror = bc + 1

    def _run(self, plan, flags, eps1=None, eps2=None, batch=None, idx=None, n_steps=1,
             counts=None, pre=None):
        if self.transport == "library" and pre is None:
            return self._lib_call(super()._run, plan, flags, eps1=eps1, eps2=eps2, batch=batch,
                                  idx=idx, n_steps=n_steps, counts=counts)
        self._closed = False

        def go(sp):
            if pre is not None:
                pre(sp)
            f = flags
            if batch is not None:
                self._pack_batch(plan, batch)
            if counts is not None:
                v = plan.views["counts"]
                v.copy_(torch.as_tensor(counts).reshape(v.shape).to(torch.float32), non_blocking=True)
                f |= _lib.OAC_STEP_COUNTS
            if idx is not None:
                self._idx.copy_(idx)
            if eps1 is not None:
                plan.views["eps1"].copy_(torch.as_tensor(eps1).reshape(plan.views["eps1"].shape))
                plan.views["eps2"].copy_(torch.as_tensor(eps2).reshape(plan.views["eps2"].shape))
            else:
                f |= _lib.OAC_STEP_DEVICE_EPS
            static = batch is None and idx is None and eps1 is None and counts is None   # ring path
            key = (id(plan), f, n_steps)
            if not (self.capture and static):
                self._steps(plan, f, n_steps, self.stream)
            elif key in self._graphs:
                self._graphs[key].replay()
            elif key not in self._eager_seen:   # first call eager (communicator warm-up)
                self._eager_seen.add(key)
                self._steps(plan, f, n_steps, self.stream)
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.stream):
                    self._steps(plan, f, n_steps, torch.cuda.current_stream(self.device))
                self._graphs[key] = g
                g.replay()
        self._on_stream(go)
        self._last_plan = plan
        if self._bc_mirror is not None:
            self._bc_mirror += n_steps
        if self._need_to_update_eval_statistics:
            self._need_to_update_eval_statistics = False
            self._fill_eval_statistics(plan)
        self._n_train_steps_total += n_steps


class DataParallelSACTrainer(_DataParallel, SACTrainer):
    """SACTrainer (trainer/trainer.py) with the data-parallel step."""


class DataParallelParticleTrainerOAC(_DataParallel, ParticleTrainerOAC):
    """ParticleTrainer (trainer/particle_trainer_oac.py) with the data-parallel step."""


class DataParallelParticleTrainer(_DataParallel, ParticleTrainer):
    """ParticleTrainer (trainer/particle_trainer.py, the p-oac recipes) with the
    data-parallel step (no alpha: the phase-0 exchange is skipped)."""


class DataParallelGaussianTrainer(_DataParallel, GaussianTrainer):
    """GaussianTrainer (trainer/gaussian_trainer.py, g-oac) with the data-parallel
    step (no alpha: the phase-0 exchange is skipped)."""
