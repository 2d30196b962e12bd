"""Drop-in ``SACTrainer`` (the trainer of ``--alg sac`` and ``--alg oac``,
/root/reference/trainer/trainer.py:14-369) running the gradient step in
liboac_amd on the GPU.

Interface kept from the reference (what rl_algorithm.py / main.py call):
constructor kwargs (trainer.py:15-31), ``train(np_batch)`` (:99-103),
``train_from_torch(batch)`` (:126), ``predict`` (:105-123), ``get_diagnostics``
(:282), ``end_epoch`` (:285), ``networks`` (:288-297), ``get_snapshot`` /
``restore_from_snapshot`` (:299-369), attributes ``policy``, ``qf1``, ``qf2``,
``target_qf1``, ``target_qf2``, ``qfs``, ``tfs``, ``log_alpha``, the four
optimizers (state_dict-compatible views) and ``deterministic``.

State lives in flat HBM arenas (params / grads / Adam m, v / targets); the
modules exposed as ``policy``, ``qf1``, ... are views into them.  One step is
one replay of a captured hipGraph of the HIP kernels (see
csrc/sac_plan.hip); nothing of the step runs in torch.
"""
import ctypes
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr
from .networks import ArenaFlattenMlp, ArenaTanhGaussianPolicy

PARAM_ORDER_POLICY = ["fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias", "last_fc.weight",
                      "last_fc.bias", "last_fc_log_std.weight", "last_fc_log_std.bias"]
PARAM_ORDER_Q = ["fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias", "last_fc.weight",
                 "last_fc.bias"]


def row_layout(obs_dim, act_dim):
    """Replay row: [obs | act | rew | term | next_obs | pad]; obs and act are
    adjacent so the critic input [obs, act] (networks.py:160) is one span."""
    off_obs, off_act = 0, obs_dim
    off_rew = obs_dim + act_dim
    off_term = off_rew + 1
    off_next = off_term + 1
    stride = (off_next + obs_dim + 3) // 4 * 4
    return dict(row_stride=stride, off_obs=off_obs, off_act=off_act, off_rew=off_rew,
                off_term=off_term, off_next_obs=off_next)


def _dims_from_state(pol_sd, q_sd):
    for sd in (pol_sd, q_sd):
        n_hidden = sum(1 for k in sd if k.startswith("fc") and k.endswith(".weight"))
        if n_hidden != 2:
            raise ValueError(f"liboac_amd implements the 2-hidden-layer MLPs of the reference "
                             f"recipes (layer_size x 2); got {n_hidden} hidden layers")
    H, Do = pol_sd["fc0.weight"].shape
    Da = pol_sd["last_fc.weight"].shape[0]
    if q_sd["fc0.weight"].shape != (H, Do + Da) or pol_sd["fc1.weight"].shape != (H, H):
        raise ValueError("policy / critic shapes are inconsistent")
    if "last_fc_log_std.weight" not in pol_sd:
        raise ValueError("only the learned-std TanhGaussianPolicy (std=None) is supported")
    return Do, Da, H, q_sd["last_fc.weight"].shape[0]


def _twin_views(arena, other, params):
    """Views of ``other`` at the offsets the ``params`` views have in ``arena``."""
    base = arena.data_ptr()
    out = []
    for p in params:
        off = (p.data_ptr() - base) // 4
        out.append(other[off:off + p.numel()].view(p.shape))
    return out


def _plain_stats(st):
    """eval_statistics with numpy scalars as Python floats (same values, same
    key order): the checkpoint then loads with torch.load(weights_only=True)."""
    from collections import OrderedDict
    if st is None:
        return st
    return OrderedDict((k, float(v) if isinstance(v, (np.generic, float, int)) else v)
                       for k, v in st.items())


class AdamStateView:
    """torch.optim.Adam-compatible ``state_dict`` over the m / v arenas.  The
    update itself is fused into the step kernels; ``step``/``zero_grad`` are
    no-ops kept for interface compatibility."""

    def __init__(self, trainer, params, m_views, v_views, lr, betas, eps, no_grad=()):
        self._t, self.params = trainer, params
        self.m, self.v = m_views, v_views
        # parameters that never receive a gradient (torch Adam keeps no state
        # for them; their m / v stay zero here, so the update is exactly 0)
        self._no_grad = set(no_grad)
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False,
                                  params=list(range(len(params))))]

    def zero_grad(self, set_to_none=True):
        pass

    def step(self, closure=None):
        pass

    def state_dict(self):
        t = self._t._n_train_steps_total
        state = {}
        if t > 0:
            for i, (m, v) in enumerate(zip(self.m, self.v)):
                if i not in self._no_grad:
                    state[i] = dict(step=t, exp_avg=m, exp_avg_sq=v)
        return dict(state=state, param_groups=[dict(g) for g in self.param_groups])

    def load_state_dict(self, sd):
        st = sd["state"]
        for i, (m, v) in enumerate(zip(self.m, self.v)):
            if i in st:
                m.copy_(torch.as_tensor(st[i]["exp_avg"]).reshape(m.shape))
                v.copy_(torch.as_tensor(st[i]["exp_avg_sq"]).reshape(v.shape))
            else:
                m.zero_()
                v.zero_()


class _ExplHandle:
    def __init__(self, handle, ws, eps, obs_np, out_np):
        self.handle, self.ws, self.eps = handle, ws, eps
        self.obs_np, self.out_np = obs_np, out_np   # views of the handle's host-coherent buffers

    def __getitem__(self, i):   # (handle, ...) unpacking of older callers
        return (self.handle, self.ws)[i]


class _Plan:
    def __init__(self, handle, ws, views, key):
        self.handle, self.ws, self.views, self.key = handle, ws, views, key


class _ArenaTrainer(object):
    """Plumbing shared by the oac_amd trainers: flat HBM arenas, per-batch-size
    launch plans (liboac_amd handles), the dedicated stream, batch packing."""

    _kind = _lib.OAC_KIND_SAC
    _q_out = 1

    def _alloc(self, Do, Da, H, device):
        L = _lib.lib()
        self.obs_dim, self.act_dim, self.hidden = Do, Da, H
        self.rows = row_layout(Do, Da)
        cfg = self._make_cfg(1)
        lay = _lib.SacLayout()
        check(L.oac_sac_query_layout(ctypes.byref(cfg), ctypes.byref(lay)))
        self.layout = lay
        z = lambda n: torch.zeros(int(n), dtype=torch.float32, device=device)
        self.params, self.grads = z(lay.params_total), z(lay.params_total)
        self.adam_m, self.adam_v = z(lay.params_total), z(lay.params_total)
        self.targets = z(lay.targets_total)
        self.alpha_state = z(16)
        self.step_state = torch.zeros(16, dtype=torch.int64, device=device)
        self.log_alpha = self.alpha_state[0:1]
        self._plans = {}
        self._bc_mirror = None   # host copy of step_state.batch_counter (drop-in path)
        self._idx = None
        self._expl = None
        self._last_plan = None
        # all library work runs on a dedicated stream: hipGraph capture needs a
        # non-default stream, and it keeps the step off torch's null stream.
        self.stream = torch.cuda.Stream(device)
        return lay

    def _next_policy_ptr(self):
        """oac_sac_buffers.next_policy: a separate network acting on next_obs
        (the g-oac / p-oac trainers' use_target_policy), or None."""
        return None

    def _on_stream(self, fn):
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            r = fn(stream_ptr(self.stream))
        cur.wait_stream(self.stream)
        return r

    # ------------------------------------------------------------ plans
    def _make_cfg(self, batch):
        c = _lib.SacConfig()
        c.kind = self._kind
        c.obs_dim, c.act_dim, c.hidden, c.q_out, c.batch = (
            self.obs_dim, self.act_dim, self.hidden, self._q_out, batch)
        c.discount, c.reward_scale, c.tau = self.discount, self.reward_scale, self.soft_target_tau
        c.policy_lr, c.qf_lr, c.beta1, c.beta2, c.adam_eps = (
            self.policy_lr, self.qf_lr, 0.9, 0.999, 1e-8)
        c.auto_alpha = int(bool(self.use_automatic_entropy_tuning))
        c.target_entropy = float(self.target_entropy)
        c.target_update_period = int(self.target_update_period)
        for k, v in self.rows.items():
            setattr(c, k, v)
        c.seed = self.seed
        c.gemm_cfg = self._gemm_cfg
        c.world_size = 1
        return c

    def _plan(self, B, replay=None, idx=None, ring_slots=0, count_state=None):
        key = (B, None if replay is None else replay.data_ptr(),
               None if idx is None else idx.data_ptr(), ring_slots,
               None if count_state is None else count_state[0].data_ptr())
        p = self._plans.get(key)
        if p is not None:
            return p
        L = _lib.lib()
        cfg = self._make_cfg(B)
        lay = _lib.SacLayout()
        check(L.oac_sac_query_layout(ctypes.byref(cfg), ctypes.byref(lay)))
        ws = torch.zeros(int(lay.workspace_floats), dtype=torch.float32, device=self.device)
        bufs = _lib.SacBuffers()
        bufs.params, bufs.grads = self.params.data_ptr(), self.grads.data_ptr()
        bufs.adam_m, bufs.adam_v = self.adam_m.data_ptr(), self.adam_v.data_ptr()
        bufs.targets = self.targets.data_ptr()
        bufs.alpha_state, bufs.step_state = self.alpha_state.data_ptr(), self.step_state.data_ptr()
        bufs.workspace = ws.data_ptr()
        bufs.replay = replay.data_ptr() if replay is not None else None
        bufs.replay_rows = replay.shape[0] if replay is not None else 0
        bufs.idx_ring = idx.data_ptr() if idx is not None else None
        bufs.ring_slots = ring_slots
        if count_state is not None:   # ReplayBufferCount device state (ring path, counts=True)
            bufs.counts, bufs.count_tags, bufs.count_epoch = (t.data_ptr() for t in count_state)
        bufs.next_policy = self._next_policy_ptr()
        h = ctypes.c_void_p()
        check(L.oac_sac_create(ctypes.byref(cfg), ctypes.byref(bufs), ctypes.byref(h)))
        views = {}
        for name, wid in _lib.WS.items():
            off, r, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            rc = L.oac_sac_workspace_view(h, wid, ctypes.byref(off), ctypes.byref(r),
                                          ctypes.byref(c))
            if rc and name in _lib.WS_OPTIONAL:
                continue
            check(rc)
            views[name] = ws[off.value:off.value + r.value * c.value].view(r.value, c.value)
        p = _Plan(h, ws, views, key)
        self._plans[key] = p
        return p

    def __del__(self):
        try:
            L = _lib.lib()
            for p in self._plans.values():   # (the drop-in plans are among them)
                L.oac_sac_destroy(p.handle)
            for e in (self._expl or {}).values():
                L.oac_expl_destroy(e.handle)
        except Exception:
            pass

    # ------------------------------------------------------------ stepping
    def _pack_batch(self, plan, batch):
        """utils/core.py:40-61: fp32 on the device, terminals as 0/1 floats."""
        X = plan.views["batch"]
        r = self.rows
        Do, Da = self.obs_dim, self.act_dim

        def put(col, n, v):
            t = torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v)
            X[:, col:col + n].copy_(t.reshape(X.shape[0], n).to(torch.float32), non_blocking=True)
        put(r["off_obs"], Do, batch["observations"])
        put(r["off_act"], Da, batch["actions"])
        put(r["off_rew"], 1, batch["rewards"])
        put(r["off_term"], 1, batch["terminals"])
        put(r["off_next_obs"], Do, batch["next_observations"])

    def _run(self, plan, flags, eps1=None, eps2=None, batch=None, idx=None, n_steps=1,
             counts=None):
        def go(sp):
            f = flags
            if batch is not None:
                self._pack_batch(plan, batch)
            if counts is not None:   # ReplayBufferCount's batch counts (counts=True trainers)
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
            if self.use_graph:
                f |= _lib.OAC_STEP_USE_GRAPH
            if n_steps == 1:
                check(_lib.lib().oac_sac_step(plan.handle, f, sp))
            else:
                check(_lib.lib().oac_sac_step_n(plan.handle, f, n_steps, sp))
        self._on_stream(go)
        self._last_plan = plan
        if self._bc_mirror is not None:
            self._bc_mirror += n_steps
        if self._need_to_update_eval_statistics:
            self._need_to_update_eval_statistics = False
            self._fill_eval_statistics(plan)
        self._n_train_steps_total += n_steps

    def train(self, np_batch):
        """trainer.py:99-103.  Accepts the reference's numpy batch dict, or the
        device batch returned by oac_amd.ReplayBuffer.random_batch (gathered
        on the GPU inside the step -- no host copy)."""
        np_batch = dict(np_batch) if not hasattr(np_batch, "device_gather") else np_batch
        if hasattr(np_batch, "device_gather"):
            self.train_device_batch(np_batch)
            return
        np_batch.pop("buffer", None)
        self.train_from_torch(np_batch)

    def train_from_torch(self, batch, eps1=None, eps2=None):
        """trainer.py:126-280 (``eps1``/``eps2``: explicit standard-normal draws
        for the two reparameterised samples, for parity runs; default: the
        device Philox stream)."""
        B = int(np.shape(batch["observations"])[0])
        plan = self._plan(B)
        self._run(plan, 0, eps1, eps2, batch=batch, counts=self._batch_counts(batch))

    def _batch_counts(self, batch):
        """batch['counts'] for trainers built with counts=True
        (particle_trainer_oac.py:220); the SAC trainer ignores it."""
        if not getattr(self, "counts", False):
            return None
        if batch.get("counts") is None:
            raise KeyError("counts=True needs batch['counts'] (ReplayBufferCount)")
        return batch["counts"]

    # host-index drop-in ring: slots of the pinned staging / device index ring
    # (a multiple of the library's 16-slot completion chunk)
    _DROPIN_SLOTS = 128

    def _dropin_plan(self, dbatch):
        """Plan + rings of the drop-in path for this (batch size, replay store)."""
        key = (dbatch.batch_size, dbatch.storage.data_ptr())
        if not hasattr(self, "_dropin"):
            self._dropin = {}
        d = self._dropin.get(key)
        if d is None:
            S, B = self._DROPIN_SLOTS, dbatch.batch_size
            ring = torch.zeros(S * B, dtype=torch.int32, device=self.device)
            d = self._plan(B, replay=dbatch.storage, idx=ring, ring_slots=S)
            # the plan's own host-coherent staging ring: at small batch the
            # step's first launch reads the indices from it directly
            check(_lib.lib().oac_sac_set_host_ring(d.handle, None))
            d.rings = (ring,)   # keep the device ring alive with the plan
            self._dropin[key] = d
        return d

    def _train_host_indices(self, dbatch):
        """rl_algorithm.py:160-167 as the reference calls it: random_batch drew
        the indices on numpy's global stream; this call stages them through a
        pinned ring and enqueues the step's launches on torch's current
        stream (ordered after replay inserts and before any later use of the
        parameters, with no host synchronisation)."""
        plan = self._dropin_plan(dbatch)
        if self._bc_mirror is None:   # device batch counter (one read after other paths ran)
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self._bc_mirror = int(self.step_state[1].item())
        idx = dbatch.host_indices
        if idx.dtype != np.int64 or not idx.flags.c_contiguous:
            idx = np.ascontiguousarray(idx, dtype=np.int64)
        check(_lib.lib().oac_sac_step_host_idx(
            plan.handle, ctypes.c_void_p(idx.ctypes.data), self._bc_mirror,
            _lib.OAC_STEP_DEVICE_EPS, stream_ptr(torch.cuda.current_stream(self.device))))
        self._bc_mirror += 1
        self._last_plan = plan
        if self._need_to_update_eval_statistics:
            self._need_to_update_eval_statistics = False
            self._fill_eval_statistics(plan)
        self._n_train_steps_total += 1

    def train_device_batch(self, dbatch, eps1=None, eps2=None):
        if (dbatch.host_indices is not None and eps1 is None
                and self._batch_counts(dbatch) is None and not getattr(self, "_no_dropin", False)):
            return self._train_host_indices(dbatch)
        B = dbatch.batch_size
        if self._idx is None or self._idx.numel() != B:
            self._idx = torch.zeros(B, dtype=torch.int32, device=self.device)
        plan = self._plan(B, replay=dbatch.storage, idx=self._idx)
        self._run(plan, _lib.OAC_STEP_GATHER, eps1, eps2, idx=dbatch.indices,
                  counts=self._batch_counts(dbatch))

    def train_from_ring(self, storage, ring, ring_slots, B, n_steps=1, count_state=None):
        """Fast path for a device-resident replay with a device index ring
        (indices drawn by the device MT19937 stream, see ReplayBuffer):
        n_steps consecutive gradient steps, each on its own minibatch --
        rl_algorithm.py's inner loop of num_trains_per_train_loop train()
        calls -- in one graph launch.  Diagnostics (on the first step after
        end_epoch in the reference) come from the last step of the call.
        counts=True trainers pass ``count_state`` =
        ReplayBufferCount.device_count_state(): each step then reads and bumps
        the drawn rows' counts on the device, exactly as random_batch does."""
        flags = _lib.OAC_STEP_GATHER
        if getattr(self, "counts", False):
            if count_state is None:
                raise ValueError("counts=True: pass count_state="
                                 "ReplayBufferCount.device_count_state()")
            if self._kind == _lib.OAC_KIND_SAC:
                raise NotImplementedError("SACTrainer has no counts targets")
            flags |= _lib.OAC_STEP_COUNTS
        else:
            count_state = None
        plan = self._plan(B, replay=storage, idx=ring, ring_slots=ring_slots,
                          count_state=count_state)
        self._run(plan, flags, n_steps=n_steps)

    def _expl_handle(self, n=1):
        """Exploration plan for n observations per call (cached per n): the
        liboac_amd handle, its workspace, a device eps slot [n, act_dim]
        (parity runs), and numpy views of the handle's host-coherent staging --
        observation rows [n, obs_dim + act_dim] and results [3, n, act_dim]
        (action | mu_E | std) -- that the kernel reads and writes itself."""
        if self._expl is None:
            self._expl = {}
        if n not in self._expl:
            L = _lib.lib()
            nf = L.oac_expl_workspace_floats_batch(n, self.obs_dim, self.act_dim, self.hidden)
            ws = torch.zeros(int(nf), dtype=torch.float32, device=self.device)
            eps = torch.zeros(n, self.act_dim, dtype=torch.float32, device=self.device)
            h = ctypes.c_void_p()
            p = self.params
            q1 = ctypes.c_void_p(p.data_ptr() + 4 * self.layout.q1_base)
            if self.layout.q2_base >= 0:     # twin critics
                check(L.oac_expl_create_batch(n, self.obs_dim, self.act_dim, self.hidden, ptr(p),
                                              q1,
                                              ctypes.c_void_p(p.data_ptr() + 4 * self.layout.q2_base),
                                              ptr(ws), ptr(self.step_state),
                                              ctypes.c_uint64(self.seed + 1), ctypes.byref(h)))
            else:                            # one shared-layer critic with K heads
                check(L.oac_expl_create_shared(n, self.obs_dim, self.act_dim, self.hidden,
                                               self._q_out, ptr(p), q1, ptr(ws),
                                               ptr(self.step_state),
                                               ctypes.c_uint64(self.seed + 1), ctypes.byref(h)))
            po, pr = ctypes.c_void_p(), ctypes.c_void_p()
            check(L.oac_expl_host_staging(h, ctypes.byref(po), ctypes.byref(pr)))
            w = self.obs_dim + self.act_dim
            obs_np = np.ctypeslib.as_array((ctypes.c_float * (n * w)).from_address(po.value))
            out_np = np.ctypeslib.as_array(
                (ctypes.c_float * (3 * n * self.act_dim)).from_address(pr.value))
            # the graph path (oac_expl_action) stages through the same buffers
            check(L.oac_expl_set_host_io(h, po, pr))
            self._expl[n] = _ExplHandle(h, ws, eps, obs_np.reshape(n, w),
                                        out_np.reshape(3, n, self.act_dim))
        return self._expl[n]


class SACTrainer(_ArenaTrainer):
    """SACTrainer (trainer/trainer.py:14) on liboac_amd."""

    def __init__(self, policy_producer, q_producer, action_space=None, discount=0.99,
                 reward_scale=1.0, policy_lr=1e-3, qf_lr=1e-3, optimizer_class=None,
                 soft_target_tau=1e-2, target_update_period=1,
                 use_automatic_entropy_tuning=True, target_entropy=None, deterministic=False,
                 device=None, seed=0, use_graph=False, gemm_cfg=-1):
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.use_automatic_entropy_tuning = use_automatic_entropy_tuning
        if use_automatic_entropy_tuning:
            if target_entropy:
                self.target_entropy = target_entropy
            else:
                self.target_entropy = -np.prod(action_space.shape).item()  # trainer.py:43-44
        else:
            self.target_entropy = 0.0
        self.soft_target_tau = soft_target_tau
        self.target_update_period = target_update_period
        self.deterministic = deterministic
        self.discount = discount
        self.reward_scale = reward_scale
        self.policy_lr, self.qf_lr = policy_lr, qf_lr
        # use_graph: each step call replayed as a captured hipGraph (n steps per
        # graph on the ring path).  Off by default: on MI355X / ROCm 7 the
        # direct launches of the same kernels measured faster (same box: ring
        # path 9,838 -> 10,456 steps/s, the counts recipes 6,444-6,565 ->
        # 7,209-7,260; the drop-in call issues its launches directly anyway)
        self.use_graph = use_graph
        self.seed = int(seed)
        self._gemm_cfg = gemm_cfg

        ref_pol = policy_producer()
        ref_q = [q_producer() for _ in range(4)]   # qf1, qf2, target_qf1, target_qf2
        pol_sd = {k: v.detach() for k, v in ref_pol.state_dict().items()}
        Do, Da, H, Q = _dims_from_state(pol_sd, ref_q[0].state_dict())
        if Q != 1:
            raise ValueError("SACTrainer critics have one output")
        lay = self._alloc(Do, Da, H, self.device)
        self.policy = ArenaTanhGaussianPolicy(self.params, 0, lay, Do, Da, H)
        self.qf1 = ArenaFlattenMlp(self.params, lay.q1_base, lay, Do, Da, H, 1)
        self.qf2 = ArenaFlattenMlp(self.params, lay.q2_base, lay, Do, Da, H, 1)
        self.target_qf1 = ArenaFlattenMlp(self.targets, 0, lay, Do, Da, H, 1)
        self.target_qf2 = ArenaFlattenMlp(self.targets, lay.q_size, lay, Do, Da, H, 1)
        self.policy.load_state_dict(pol_sd)
        for mod, ref in zip((self.qf1, self.qf2, self.target_qf1, self.target_qf2), ref_q):
            mod.load_state_dict({k: v.detach() for k, v in ref.state_dict().items()})
        self.policy.oac_trainer = self
        self.qfs = [self.qf1, self.qf2]
        self.tfs = [self.target_qf1, self.target_qf2]
        # optimizer views (the m / v arenas share the params layout)
        tw = lambda other, mod: _twin_views(self.params, other, list(mod.parameters()))
        self.policy_optimizer = AdamStateView(self, list(self.policy.parameters()),
                                              tw(self.adam_m, self.policy),
                                              tw(self.adam_v, self.policy), policy_lr,
                                              (0.9, 0.999), 1e-8)
        self.qf1_optimizer = AdamStateView(self, list(self.qf1.parameters()),
                                           tw(self.adam_m, self.qf1), tw(self.adam_v, self.qf1),
                                           qf_lr, (0.9, 0.999), 1e-8)
        self.qf2_optimizer = AdamStateView(self, list(self.qf2.parameters()),
                                           tw(self.adam_m, self.qf2), tw(self.adam_v, self.qf2),
                                           qf_lr, (0.9, 0.999), 1e-8)
        self.alpha_optimizer = AdamStateView(self, [self.log_alpha], [self.alpha_state[1:2]],
                                             [self.alpha_state[2:3]], policy_lr, (0.9, 0.999), 1e-8)
        self.eval_statistics = OrderedDict()
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True

    # ------------------------------------------------------------ diagnostics
    def _fill_eval_statistics(self, plan):
        v = {k: t.detach().to("cpu").numpy() for k, t in plan.views.items()
             if k in ("q1", "q2", "y", "logp1", "head1", "sqe1", "sqe2", "qnew")}
        Da = self.act_dim
        q1, q2 = v["q1"], v["q2"]
        st = OrderedDict()
        qs = np.stack([q1, q2], axis=0)
        st["QF mean"] = np.mean(qs, axis=0).mean()
        st["QF std"] = np.std(qs, axis=0).mean()
        l1, l2 = np.float32(np.mean(v["sqe1"])), np.float32(np.mean(v["sqe2"]))
        st["QF1 Loss"] = l1
        st["QF2 Loss"] = l2
        st["Q Loss"] = np.float32(l1 + l2)
        st["Policy Loss"] = np.mean(v["logp1"] - v["qnew"])       # trainer.py:236 (no alpha)
        mean = v["head1"][:, :Da]
        log_std = np.clip(v["head1"][:, Da:], -20, 2)
        for name, arr in (("Q1 Predictions", q1), ("Q2 Predictions", q2), ("Q Targets", v["y"]),
                          ("Log Pis", v["logp1"]), ("Policy mu", mean),
                          ("Policy log std", log_std)):
            st[name + " Mean"] = np.mean(arr)
            st[name + " Std"] = np.std(arr)
            st[name + " Max"] = np.max(arr)
            st[name + " Min"] = np.min(arr)
        if self.use_automatic_entropy_tuning:
            a = self.alpha_state.detach().cpu().numpy()
            st["Alpha"] = float(a[3])
            st["Alpha Loss"] = float(a[4])
        self.eval_statistics = st

    def get_diagnostics(self):
        return self.eval_statistics

    def end_epoch(self, epoch):
        self._need_to_update_eval_statistics = True

    # ------------------------------------------------------------ misc API
    def predict(self, obs, action, upper_bound=True, beta_UB=4.46, both_values=False):
        """trainer.py:105-123: Q_UB = (Q1+Q2)/2 + beta_UB |Q1-Q2|/2, both critics
        in one oac_critic_eval launch; differentiable w.r.t. obs and action
        (the reference's exploration takes autograd.grad of it)."""
        from .networks import _as_input, critics_apply
        obs, action = _as_input(obs, self.device), _as_input(action, self.device)
        if obs.dim() == 1:
            obs, action = obs.unsqueeze(0), action.unsqueeze(0)
        q = critics_apply([self.qf1, self.qf2], obs, action)
        q1, q2 = q[:, 0:1], q[:, 1:2]
        mu, sigma = (q1 + q2) / 2.0, torch.abs(q1 - q2) / 2.0
        if both_values:
            return mu, sigma
        if not upper_bound:
            return mu
        return mu + beta_UB * sigma

    @property
    def networks(self):
        return [self.policy, self.qf1, self.qf2, self.target_qf1, self.target_qf2]

    def get_snapshot(self):
        snapshot = dict(
            policy_state_dict=self.policy.state_dict(),
            policy_optim_state_dict=self.policy_optimizer.state_dict(),
            qf1_state_dict=self.qf1.state_dict(),
            qf1_optim_state_dict=self.qf1_optimizer.state_dict(),
            target_qf1_state_dict=self.target_qf1.state_dict(),
            qf2_state_dict=self.qf2.state_dict(),
            qf2_optim_state_dict=self.qf2_optimizer.state_dict(),
            target_qf2_state_dict=self.target_qf2.state_dict(),
            eval_statistics=_plain_stats(self.eval_statistics),
            _n_train_steps_total=self._n_train_steps_total,
            _need_to_update_eval_statistics=self._need_to_update_eval_statistics,
        )
        if self.use_automatic_entropy_tuning:
            snapshot["log_alpha"] = self.log_alpha
            snapshot["alpha_optim_state_dict"] = self.alpha_optimizer.state_dict()
        return snapshot

    def restore_from_snapshot(self, ss):
        self.policy.load_state_dict(ss["policy_state_dict"])
        self.policy_optimizer.load_state_dict(ss["policy_optim_state_dict"])
        for name in ("qf1", "qf2"):
            getattr(self, name).load_state_dict(ss[f"{name}_state_dict"])
            getattr(self, f"{name}_optimizer").load_state_dict(ss[f"{name}_optim_state_dict"])
            getattr(self, f"target_{name}").load_state_dict(ss[f"target_{name}_state_dict"])
        if self.use_automatic_entropy_tuning:
            self.log_alpha.copy_(torch.as_tensor(ss["log_alpha"]).reshape(1))
            self.alpha_optimizer.load_state_dict(ss["alpha_optim_state_dict"])
            self.alpha_state[3] = torch.exp(self.log_alpha[0])
        self.eval_statistics = ss["eval_statistics"]
        self._n_train_steps_total = int(ss["_n_train_steps_total"])
        self._need_to_update_eval_statistics = ss["_need_to_update_eval_statistics"]
        self.step_state[0] = self._n_train_steps_total

    # ------------------------------------------------------------ exploration
