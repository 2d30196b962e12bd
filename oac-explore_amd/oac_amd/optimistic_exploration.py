"""Drop-in ``get_optimistic_exploration_action``
(/root/reference/optimistic_exploration.py:7-11) -- the OAC action shift,
computed by liboac_amd in one launch (csrc/expl_plan.hip, expl_split.hip), for
twin critics (SACTrainer) or one shared-layer critic with K heads
(ParticleTrainerOAC, share_layers: Q_UB = mean_k + beta_UB std_k).

Same signature and return value as the reference: ``(action float32[Da], {})``
for a 1-D observation.  ``get_optimistic_exploration_actions`` is the
vectorised-rollout extension: N observations [N, Do] in one launch
sequence, each row exactly as a single call.  ``policy`` must be the policy of an oac_amd trainer
(its parameters live in the trainer's HBM arena, which the kernels read in
place); there is no torch/CPU fallback.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


def _owner(policy, qfs, trainer, hyper_params):
    """The oac_amd trainer whose arena holds ``policy`` and ``qfs``.  Twin
    critics take the try branch of optimistic_exploration.py:40-46 whatever
    share_layers says; one shared-layer critic with K heads takes the except
    branch (:47-56), which only works with share_layers=True.  With trainer
    (--trainer_UB, :38-39) Q_UB is trainer.predict: for SACTrainer the same
    twin bound (trainer/trainer.py:105-123), for the P-OAC ParticleTrainer the
    head sorted at its delta_index (particle_trainer_oac.py:147-167)."""
    t = getattr(policy, "oac_trainer", None)
    if t is None:
        raise TypeError("get_optimistic_exploration_action: policy is not an oac_amd policy "
                        "(build the trainer with oac_amd.SACTrainer / ParticleTrainerOAC)")
    if qfs is not None and (len(qfs) != len(t.qfs) or any(a is not b for a, b in zip(qfs, t.qfs))):
        raise NotImplementedError("qfs must be the critics of the trainer that owns the policy")
    twin = t.layout.q2_base >= 0
    if trainer is not None:
        if trainer is not t:
            raise NotImplementedError("trainer_UB must be the trainer that owns the policy")
        from .particle_trainer_oac import ParticleTrainer as _ParticleTrainerOAC
        if not twin and not isinstance(t, _ParticleTrainerOAC):
            # the reference fails here too: particle_trainer.py:157 / gaussian_trainer.py
            # predict() take no upper_bound / beta_UB keywords (optimistic_exploration.py:39)
            raise TypeError("trainer_UB needs SACTrainer (twin critics) or the P-OAC "
                            "ParticleTrainer of particle_trainer_oac.py (sorted-head upper "
                            "bound, :147-167); this trainer's predict() has no upper_bound")
        if not twin and getattr(t, "delta_index", None) is None:
            raise ValueError("trainer_UB with the P-OAC ParticleTrainer needs its delta_index: "
                             "delta must be a quantile level in (0, 1) "
                             f"(particle_trainer_oac.py:60-67), got delta={t.delta}")
    elif not twin and not hyper_params.get("share_layers", False):
        raise ValueError("one critic with K heads needs hyper_params['share_layers'] = True "
                         "(the reference's except branch fails without it)")
    return t


def get_optimistic_exploration_action(ob_np, policy=None, qfs=None, trainer=None,
                                      hyper_params=None, deterministic=False, eps=None,
                                      return_info=False):
    """optimistic_exploration.py:7-11 / 14-109 (stochastic branch).

    ``trainer`` (--trainer_UB): for SACTrainer the same Q_UB = mean +
    beta_UB*|Q1-Q2|/2 as the qfs branch (trainer/trainer.py:105-123); for the
    P-OAC ParticleTrainer the head sorted at its delta_index
    (particle_trainer_oac.py:147-167, oac_expl_set_ub_index).  ``eps`` (float32[Da]) replaces the device Philox draw for parity
    runs; ``return_info`` adds mu_E / std / grad to the info dict."""
    if deterministic:
        raise NotImplementedError("the deterministic OAC variant is unreachable from rollout() "
                                  "(SURVEY 8a quirk Q7) and not implemented")
    if eps is None and not return_info and not _USE_GRAPH:
        return _action_now(ob_np, policy, qfs, trainer, hyper_params), {}
    assert np.ndim(ob_np) == 1
    t = _owner(policy, qfs, trainer, hyper_params)
    a, info = _actions(t, np.asarray(ob_np)[None, :], hyper_params,
                       None if eps is None else np.asarray(eps, np.float32)[None, :], return_info,
                       trainer is not None)
    return a[0], {k: v[0] for k, v in info.items()}


# the per-environment-step call (path_collector.py:219-220) validates the same
# (policy, qfs, trainer, share_layers) every step: the validated combinations
# are remembered on the policy object itself, so nothing outlives the trainer
# (the policy already references its trainer), each with what the call needs
# ready-made -- the library function, the handle, the staging views, the
# device index.  A cached qfs key is ids of the owning trainer's own critics,
# which that trainer keeps alive, so an id in it cannot be reused by another
# object while the entry exists.  (The Python side of a call: 1.96 us of a
# 25.9 us call with the owner check cached only, 1.04 of 25.3 with the whole
# call record cached; the library call alone 24.2 us: tools/r6/expl_py.py.)
_CACHE_ATTR = "_oac_expl_validated"


class _Fast:
    __slots__ = ("t", "e", "obs", "out", "fn", "handle", "dev", "heads", "trainer_ub")

    def __init__(self, t, trainer_ub):
        self.t = t
        self.e = e = t._expl_handle(1)
        self.obs = e.obs_np[0, :t.obs_dim]        # fp32 view of the staging row
        self.out = e.out_np[0, 0]                 # the action row of the results
        self.fn = _lib.lib().oac_expl_action_now
        self.handle = e.handle
        self.dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
        self.heads = t.layout.q2_base < 0         # K heads: mean + beta std, or the sorted head
        self.trainer_ub = trainer_ub


def _action_now(ob_np, policy, qfs, trainer, hyper_params):
    """The single-observation Philox call on its shortest host path: cached
    owner validation and call record, the raw current-stream handle, one C
    call."""
    share = bool(hyper_params.get("share_layers", False))
    key = (trainer is not None, None if qfs is None else tuple(map(id, qfs)), share)
    seen = policy.__dict__.get(_CACHE_ATTR)
    f = seen.get(key) if seen is not None else None
    if f is None or (trainer is not None and trainer is not f.t):
        t = _owner(policy, qfs, trainer, hyper_params)   # (raises for a foreign trainer)
        if seen is None:
            seen = policy.__dict__[_CACHE_ATTR] = {}
        f = seen[key] = _Fast(t, trainer is not None)
    if (ob_np.ndim if type(ob_np) is np.ndarray else np.ndim(ob_np)) != 1:
        raise AssertionError("get_optimistic_exploration_action: one observation (1-D)")
    if f.heads:
        check(_lib.lib().oac_expl_set_ub_index(f.handle, int(f.t.delta_index) if f.trainer_ub else -1))
    f.obs[:] = ob_np                                  # float64 observation -> fp32 row
    rc = f.fn(f.handle, None, float(hyper_params["beta_UB"]), float(hyper_params["delta"]),
              torch._C._cuda_getCurrentRawStream(f.dev))
    if rc:
        check(rc)
    return f.out.copy()


def get_optimistic_exploration_actions(obs_np, policy=None, qfs=None, trainer=None,
                                       hyper_params=None, eps=None, return_info=False):
    """Vectorised get_optimistic_exploration_action: ``obs_np`` [N, Do] (one
    row per parallel environment) -> (actions float32 [N, Da], info).  The
    Philox draws of a call use one counter value (row r takes elements
    r*Da .. r*Da+Da-1 of the stream); ``eps`` [N, Da] replaces them."""
    assert np.ndim(obs_np) == 2
    t = _owner(policy, qfs, trainer, hyper_params)
    return _actions(t, np.asarray(obs_np), hyper_params,
                    None if eps is None else np.asarray(eps, np.float32), return_info,
                    trainer is not None)


_USE_GRAPH = os.environ.get("OAC_EXPL_GRAPH", "0") == "1"


def _actions(t, obs, hyper_params, eps, return_info, trainer_ub=False):
    """One launch on torch's current stream: the kernel reads the observations
    from and writes the results to the handle's host-coherent staging, and the
    call returns when its completion word lands (oac_expl_action_now).
    OAC_EXPL_GRAPH=1: the captured-graph path instead (oac_expl_action: upload,
    kernel and download replayed, then a stream synchronisation)."""
    n = obs.shape[0]
    e = t._expl_handle(n)
    if t.layout.q2_base < 0:   # K heads: mean + beta std, or trainer.predict's sorted head
        check(_lib.lib().oac_expl_set_ub_index(e.handle, int(t.delta_index) if trainer_ub else -1))
    e.obs_np[:, :t.obs_dim] = obs                 # float64 observations -> fp32 rows
    # torch's current stream: every trainer call leaves it behind its updates
    # (_on_stream; the drop-in step runs on it), so the weights read are the
    # latest, with no cross-stream join on this path
    s = torch.cuda.current_stream(t.device)
    ed = None
    if eps is not None:
        e.eps.copy_(torch.from_numpy(np.ascontiguousarray(eps, np.float32)).reshape(e.eps.shape))
        ed = e.eps
    beta, delta = float(hyper_params["beta_UB"]), float(hyper_params["delta"])
    if _USE_GRAPH:
        check(_lib.lib().oac_expl_action(e.handle, ptr(ed), beta, delta, None, None, None, None,
                                         stream_ptr(s)))
        s.synchronize()
    else:
        check(_lib.lib().oac_expl_action_now(e.handle, ptr(ed), beta, delta, stream_ptr(s)))
    res = e.out_np
    info = {}
    if return_info:
        info = dict(mu_E=res[1].copy(), std=res[2].copy())
    return res[0].copy(), info
