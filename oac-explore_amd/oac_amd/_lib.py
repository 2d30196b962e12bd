"""ctypes binding of liboac_amd.so (the C ABI declared in include/oac_amd.h).

The library is built in-tree (``make -C oac-explore_amd`` or
``__graft_entry__.build()``).  There is no fallback: if the shared library is
missing or cannot be loaded, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# OAC_LIB: another in-tree build of the same library (same-box A/B runs of a
# kernel change, e.g. tools/ab_lib.sh); the default is the package's own
_DEFAULT_LIB = os.path.join(HERE, "liboac_amd.so")
LIB_PATH = os.environ.get("OAC_LIB") or _DEFAULT_LIB

OAC_KIND_SAC = 0
OAC_KIND_PARTICLE = 1
OAC_KIND_GAUSS = 2
OAC_KIND_PARTICLE_UB = 3

OAC_STEP_GATHER = 1
OAC_STEP_DEVICE_EPS = 2
OAC_STEP_USE_GRAPH = 4
OAC_STEP_COUNTS = 8

OAC_DP_FORCE = 1
OAC_DP_OVERLAP = 2

# oac_sac_trace bits
TRACE = dict(direct=1, direct_big=2, batch_copy=4, qdot=8, wl_targets=16, split_phase1=32,
             fused=64, exchange=128, la_adam=256, head_dh2=512)

# oac_allreduce_fn: int (*)(void* ctx, float* buf, int64_t n, void* stream)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_void_p)

# public workspace ids (enum oac_ws_buffer)
WS = {name: i for i, name in enumerate([
    "batch", "eps1", "eps2", "head1", "head2", "act1", "act2", "logp1", "logp2",
    "q1", "q2", "qn1", "qn2", "tq1", "tq2", "y", "sqe1", "sqe2", "qnew", "counts",
    "head3", "act3", "logp_part", "h2q1", "h2q2", "h1p", "h2p"])}
# non-default kernel / schedule choices (enum oac_tuning_key; A/B runs and the
# alternative-kernel parity tests): set_tuning(bwdp_cfg=9, ...) before the
# trainers that should use them create their plans; 0 restores a default
TUNE = {name: i for i, name in enumerate([
    "bwdp_cfg", "fwd_tile_m", "fwd_tile_n", "fwd_nb", "split_adam", "dh2_targets", "head_cc",
    "splits_q1", "splits_q0", "splits_ph", "splits_p1", "splits_p0", "debug_cfg",
    "ring_direct", "ring_prefetch", "la_adam", "head_dh2"])}


def set_tuning(**kw):
    for k, v in kw.items():
        check(lib().oac_tuning_set(TUNE[k], int(v)))


def set_tuning_spec(spec):
    """set_tuning from "key=value,key=value" (tools' A/B scripts)."""
    if spec:
        set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in spec.split(",") if kv)})


# diagnostic views a library build may predate (skipped when it rejects the id)
WS_OPTIONAL = ("h1p", "h2p")


class SacConfig(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int), ("obs_dim", ctypes.c_int), ("act_dim", ctypes.c_int),
        ("hidden", ctypes.c_int), ("q_out", ctypes.c_int), ("batch", ctypes.c_int),
        ("discount", ctypes.c_float), ("reward_scale", ctypes.c_float), ("tau", ctypes.c_float),
        ("policy_lr", ctypes.c_double), ("qf_lr", ctypes.c_double), ("beta1", ctypes.c_double),
        ("beta2", ctypes.c_double), ("adam_eps", ctypes.c_double),
        ("auto_alpha", ctypes.c_int), ("target_entropy", ctypes.c_float),
        ("target_update_period", ctypes.c_int), ("row_stride", ctypes.c_int),
        ("off_obs", ctypes.c_int), ("off_act", ctypes.c_int), ("off_rew", ctypes.c_int),
        ("off_term", ctypes.c_int), ("off_next_obs", ctypes.c_int),
        ("seed", ctypes.c_uint64), ("gemm_cfg", ctypes.c_int), ("world_size", ctypes.c_int),
        ("std_bound", ctypes.c_float), ("std_init", ctypes.c_float),
        ("std_soft_update", ctypes.c_int), ("std_soft_prob", ctypes.c_float),
        ("mean_update", ctypes.c_int), ("delta_index", ctypes.c_int),
        ("rescale_spread", ctypes.c_float), ("freeze_q_bias", ctypes.c_int),
    ]


class SacLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "pol_fc0_w", "pol_fc0_b", "pol_fc1_w", "pol_fc1_b", "pol_head_w", "pol_head_b", "pol_size",
        "q_fc0_w", "q_fc0_b", "q_fc1_w", "q_fc1_b", "q_last_w", "q_last_b", "q_size",
        "q1_base", "q2_base", "n_critics", "params_total", "targets_total", "workspace_floats",
        "tpol_base")]


class SacBuffers(ctypes.Structure):
    _fields_ = [
        ("params", ctypes.c_void_p), ("grads", ctypes.c_void_p), ("adam_m", ctypes.c_void_p),
        ("adam_v", ctypes.c_void_p), ("targets", ctypes.c_void_p),
        ("alpha_state", ctypes.c_void_p), ("step_state", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p), ("replay", ctypes.c_void_p),
        ("replay_rows", ctypes.c_int64), ("idx_ring", ctypes.c_void_p),
        ("ring_slots", ctypes.c_int),
        ("counts", ctypes.c_void_p), ("count_tags", ctypes.c_void_p),
        ("count_epoch", ctypes.c_void_p), ("next_policy", ctypes.c_void_p),
    ]


_LIB = None

_SIGS = {
    "oac_last_error": (ctypes.c_char_p, []),
    "oac_abi_version": (ctypes.c_int, []),
    "oac_sac_query_layout": (ctypes.c_int, [ctypes.POINTER(SacConfig), ctypes.POINTER(SacLayout)]),
    "oac_sac_create": (ctypes.c_int, [ctypes.POINTER(SacConfig), ctypes.POINTER(SacBuffers),
                                      ctypes.POINTER(ctypes.c_void_p)]),
    "oac_sac_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "oac_sac_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oac_sac_step_n": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p]),
    "oac_sac_step_phase": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]),
    "oac_sac_set_host_ring": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "oac_sac_host_ring": (ctypes.c_void_p, [ctypes.c_void_p]),
    "oac_sac_step_host_idx": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_int, ctypes.c_void_p]),
    "oac_sac_stage_host_idx": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_void_p]),
    "oac_sac_set_step_graph": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "oac_sac_set_allreduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int]),
    "oac_sac_trace": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oac_rccl_unique_id": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p]),
    "oac_rccl_create": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "oac_rccl_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "oac_rccl_allreduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p]),
    "oac_sac_workspace_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_int64),
                                              ctypes.POINTER(ctypes.c_int64),
                                              ctypes.POINTER(ctypes.c_int64)]),
    "oac_sac_launch_count": (ctypes.c_int, [ctypes.c_void_p]),
    "oac_sac_cache_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "oac_tuning_set": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "oac_sac_set_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oac_sac_read_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int64), ctypes.c_int]),
    "oac_sac_read_launch_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "oac_critic_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "oac_policy_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "oac_mt_seed_host": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_void_p]),
    "oac_replay_sample_indices": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    "oac_replay_gather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "oac_replay_insert": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p]),
    "oac_replay_counts_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int, ctypes.c_int32, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "oac_replay_priority_scratch_doubles": (ctypes.c_int64, [ctypes.c_int64]),
    "oac_replay_priority_sample": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p]),
    "oac_adam_polyak": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                       ctypes.c_float, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "oac_expl_workspace_floats": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "oac_expl_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "oac_expl_workspace_floats_batch": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                         ctypes.c_int]),
    "oac_expl_create_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "oac_expl_create_shared": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "oac_expl_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "oac_expl_obs_slot": (ctypes.c_void_p, [ctypes.c_void_p]),
    "oac_expl_action": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                       ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "oac_expl_outputs": (ctypes.c_void_p, [ctypes.c_void_p]),
    "oac_expl_set_host_io": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "oac_expl_set_ub_index": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "oac_expl_host_staging": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "oac_expl_action_now": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_void_p]),
}

# every symbol include/oac_amd.h declares (checked by tests/test_abi.py)
EXPORTED = sorted(_SIGS)


def lib():
    """Load liboac_amd.so (after torch, so the HIP runtime torch already
    loaded -- same soname libamdhip64.so.7 -- is the one the library binds)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is not built: run `make -C oac-explore_amd` (or "
            "__graft_entry__.build()).  There is no CPU fallback for the OAC hot path.")
    import torch  # noqa: F401  (HIP runtime first)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if LIB_PATH != _DEFAULT_LIB and not hasattr(L, name):
            continue   # an OAC_LIB A/B build of an older tree: its entry points only
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.oac_abi_version() != 3:
        raise RuntimeError("liboac_amd ABI version mismatch")
    _LIB = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().oac_last_error().decode(errors="replace")
        raise RuntimeError(f"liboac_amd: {msg}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
