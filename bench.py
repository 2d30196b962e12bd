"""OAC gradient-step benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

Workload (BASELINE.json configs[1], the metric's config): SAC/OAC trainer
step, Humanoid-v2 dims (obs 376, act 17), 2x256 MLPs, batch 256 per rank,
replay 1e6 transitions resident in HBM, synthetic data (random-init weights,
N(0,1) observations, U(-1,1) actions, N(0,1) rewards, Bernoulli(0.01)
terminals).  A "step" is one full gradient step: device index draw (MT19937,
numpy-exact), replay gather, policy/critic forward + backward, alpha, the
three Adam updates and Polyak -- one hipGraph replay.

N > 1 (torchrun, one process per GPU): data parallel, replay sharded per
rank, gradients all-reduced over RCCL (see oac_amd/dp.py); value = gradient
steps of batch B processed by all ranks per second (weak scaling).
"""
import argparse
import ctypes
import gc
import json
import os
import sys
import time


def _pin_host_threads(per_rank=4):
    """Keep this rank's host threads on `per_rank` fixed cores of the ones it
    may use (rank r: the r-th slice, by LOCAL_RANK), set before torch starts
    its threads so they all inherit it.  The timed loop is host-issued
    launches; left to migrate, the driver-shaped line spread 11,064-11,416
    steps/s over six runs on one box, pinned to 8 cores 11,491-11,544
    (tools/r6/variance.sh); 2 / 4 / 8 / 16 cores measured 11,536 / 11,526 /
    11,491 / 11,420 (means of three, tools/r6/pinsize.sh).  Not in the `--gpus N` launcher process (its
    ranks take their own slices) and not with --no-pin; returns the cores the
    process had (the CPU baselines' fresh process starts on them)."""
    argv = sys.argv[1:]
    gpus = 1
    for i, a in enumerate(argv):
        v = a.split("=", 1)[1] if a.startswith("--gpus=") else (
            argv[i + 1] if a == "--gpus" and i + 1 < len(argv) else None)
        if v is not None and v.isdigit():
            gpus = int(v)
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    if "--no-pin" in argv or ("WORLD_SIZE" not in os.environ and gpus > 1):
        return allowed
    lr = int(os.environ.get("LOCAL_RANK", "0") or 0)
    if len(allowed) >= per_rank * (lr + 1):
        os.sched_setaffinity(0, allowed[per_rank * lr:per_rank * (lr + 1)])
    return allowed


# (as the benchmark process only: a process that imports bench -- the tests,
# tools/launch_times.py -- keeps its threads where they are)
_HOST_CPUS = _pin_host_threads() if __name__ == "__main__" else None

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))

FLOP_PER_SAMPLE = 4_377_600        # algorithmic GEMM FLOPs per sample (SAC, Humanoid)
# what the build's MFMAs execute per sample (SAC, Humanoid): the fresh-action
# critics reuse the obs projection W0[:, :376] obs of Q(obs, a) / TQ(next_obs)
# and add a rank-17 action update, so two 376 x 256 products per sample of the
# 8d count are not executed (1,996,288 MAC against 2,188,800: 8.8 % fewer)
EXEC_FLOP_PER_SAMPLE = 3_992_576
FLOP_PER_SAMPLE_POAC_ANT = 1_792_512   # P-OAC K=10, Ant dims
GATHER_BYTES_PER_SAMPLE = 3_081 + 4
ADAM_BYTES_PER_STEP = 18_142_244
PEAK_FP32_TFLOPS = 157.3           # MI355X fp32 MFMA dense peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=640)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--obs-dim", type=int, default=376)
    ap.add_argument("--act-dim", type=int, default=17)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--replay", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pin", action="store_true",
                    help="leave the host threads unpinned (bench.py pins each rank to 4 cores)")
    ap.add_argument("--cpu-baseline-only", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the exploration and g-oac legs (profiling runs: keeps the "
                         "per-kernel statistics to the headline step)")
    ap.add_argument("--timing-steps", type=int, default=50)
    ap.add_argument("--gemm-cfg", type=int, default=-1)
    ap.add_argument("--mode", choices=("dropin", "ring"), default="dropin",
                    help="dropin: the reference loop (random_batch + train per step, "
                         "rl_algorithm.py:160-167); ring: train_from_ring with the device "
                         "index stream, --steps-per-launch steps per graph")
    ap.add_argument("--selftest-launcher", action="store_true",
                    help="CPU-only check of the --gpus N rank launcher (gloo all-reduce)")
    ap.add_argument("--steps-per-launch", type=int, default=64,
                    help="gradient steps per graph launch (1 = one graph per step); the "
                         "default is the device index ring's refill period, i.e. one "
                         "rl_algorithm train-loop stretch of 64 train() calls per launch")
    return ap.parse_args()


def synthetic_rows(n, rows, obs_dim, act_dim, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.zeros(n, rows["row_stride"], dtype=torch.float32, device=device)
    o, a = rows["off_obs"], rows["off_act"]
    out[:, o:o + obs_dim] = torch.randn(n, obs_dim, generator=g, device=device)
    out[:, a:a + act_dim] = torch.rand(n, act_dim, generator=g, device=device) * 2 - 1
    out[:, rows["off_rew"]] = torch.randn(n, generator=g, device=device)
    out[:, rows["off_term"]] = (torch.rand(n, generator=g, device=device) < 0.01).float()
    no = rows["off_next_obs"]
    out[:, no:no + obs_dim] = torch.randn(n, obs_dim, generator=g, device=device)
    return out


class Space:
    def __init__(self, n):
        self.shape = (n,)
        self.low = np.zeros(n, np.float32)


def force_dp():
    """OAC_BENCH_FORCE_DP=1 (under torchrun): the data-parallel step even at
    one rank -- phase split, unfused Adam, RCCL all-reduces in the graph --
    to measure what the DP structure costs apart from the link latency."""
    return os.environ.get("OAC_BENCH_FORCE_DP") == "1"


def build(args, rank, world, device):
    import oac_amd
    from oac_amd import DeviceIndexStream, ReplayBuffer, SACTrainer
    torch.manual_seed(0)   # identical init on every rank
    hid = [args.hidden, args.hidden]
    pp = oac_amd.get_policy_producer(args.obs_dim, args.act_dim, hid, device=device)
    qp = oac_amd.get_q_producer(args.obs_dim, args.act_dim, hid, device=device)
    kw = dict(action_space=Space(args.act_dim), discount=0.99, reward_scale=1.0,
              policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3, target_update_period=1,
              use_automatic_entropy_tuning=True, device=device, seed=2 + 1000 * rank,
              gemm_cfg=args.gemm_cfg)
    if world > 1 or force_dp():
        from oac_amd.dp import DataParallelSACTrainer
        tr = DataParallelSACTrainer(pp, qp, **kw)
    else:
        tr = SACTrainer(pp, qp, **kw)
    # the reference SAC / OAC recipes use the plain ReplayBuffer (main.py:179-183)
    rb = ReplayBuffer(args.replay, args.obs_dim, args.act_dim, device=device)
    rb.load_transitions(synthetic_rows(args.replay, rb.rows, args.obs_dim, args.act_dim,
                                       device, seed=rank))
    stream = DeviceIndexStream(rb, args.batch, chunk=64, seed=1 + rank)
    return tr, rb, stream


def step_fn(tr, rb, stream, B, n=1):
    """One call = n consecutive gradient steps (n divides the 64-step index
    chunk), each on its own minibatch; n > 1 replays one n-step graph."""
    def step():
        stream.before_step(n)
        tr.train_from_ring(rb._storage, stream.ring, stream.slots, B, n_steps=n)
    return step


def timed(run, steps, warmup, world, device):
    """run(warmup), then time run(steps) between barriers + device syncs;
    the max over ranks."""
    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()
    # host jitter: no Python garbage collection inside the timed region (the
    # driver times 20 steps = ~2 ms; a collection pause is a visible share),
    # collected before the warm-up (which re-warms the host caches)
    gc.collect()
    gc_on = gc.isenabled()
    gc.disable()
    try:
        run(warmup)
        barrier()
        t0 = time.perf_counter()
        run(steps)
        barrier()
        el = time.perf_counter() - t0
    finally:
        if gc_on:
            gc.enable()
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return el


def dropin_run(tr, rb, B):
    def run(k):
        for _ in range(k):
            train_data = rb.random_batch(B)
            train_data["buffer"] = rb
            tr.train(train_data)
    return run


def roofline_of(kt, flop_per_sample, B, n, traffic_key=None, exec_flop_per_sample=None):
    """The dominant kernel family's roofline: ALGORITHMIC flops per launch
    (SURVEY 8d per-sample figure x samples per step / GEMM launches per step)
    over the average launch duration measured live with dispatch events
    (kernel_timing: the begin->end interval of each launch, as rocprofv3's
    kernel trace reports it; the same command under rocprofv3 is committed
    in profiles/)."""
    gk = kt["gemm_grouped"]
    fpl = flop_per_sample * B * n / max(gk["launches"], 1)
    ach = fpl / (gk["avg_us"] * 1e-6) / 1e12
    out = {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_FP32_TFLOPS,
           "unit": "TFLOP/s", "frac": round(ach / PEAK_FP32_TFLOPS, 4),
           "traffic": load_traffic(traffic_key or B), "flops_per_launch": round(fpl),
           "avg_launch_us": round(gk["avg_us"], 3), "launches_per_step": gk["launches"] / n,
           "duration_source": "hipExtLaunchKernel dispatch events, %d steps" % n}
    prof = rocprof_gemm_avg(traffic_key or B)
    if prof is not None:   # the same figure from the committed rocprofv3 statistics
        us, path = prof
        a2 = fpl / (us * 1e-6) / 1e12
        out["rocprof"] = {"avg_launch_us": us, "achieved": round(a2, 3),
                          "frac": round(a2 / PEAK_FP32_TFLOPS, 4), "source": path,
                          "note": "a profiled run of the same command: under rocprofv3 the "
                                  "direct-launch step is host-bound (kernels start after host "
                                  "gaps), and back to back it stamps a kernel's start at the "
                                  "previous kernel's end (the launch edge inside the duration); "
                                  "the dispatch events above are the timed process's own "
                                  "(DESIGN.md section 4)"}
    if exec_flop_per_sample:
        out["executed_flops_per_launch"] = round(exec_flop_per_sample * B * n / max(gk["launches"], 1))
        out["note"] = ("numerator = SURVEY 8d algorithmic GEMM FLOPs; the MFMAs execute %.1f %% fewer "
                       "(obs projections reused by the fresh-action critics)"
                       % (100.0 * (1 - exec_flop_per_sample / flop_per_sample)))
    return out


def hbm_legs(kt, B, n):
    """SURVEY 8d HBM sub-roofline of the step's own gather launches (the
    materialised replay gather: B x (3,085 read + 3,081 written) bytes per
    launch), from the same dispatch events as the GEMM roofline."""
    out = {}
    ga = kt["gather"]
    if ga["launches"]:
        gb = (GATHER_BYTES_PER_SAMPLE + 3_081) * B * n / ga["launches"]
        rate = gb / (ga["avg_us"] * 1e-6) / 1e9
        out["gather"] = {"GBps": round(rate, 1), "bytes_per_launch": round(gb),
                         "avg_launch_us": round(ga["avg_us"], 3), "launches_per_step": ga["launches"] / n,
                         "frac_of_hbm_peak": round(rate / PEAK_HBM_GBS, 4)}
    return out


def standalone_hbm(rb, device, B=4096, reps=50):
    """SURVEY 8d "sub-kernels measured separately against HBM": the replay
    gather (oac_replay_gather of B random rows of the resident 1e6-row replay,
    B x (3,085 + 3,081) algorithmic bytes) and one SAC step's Adam + Polyak
    (oac_adam_polyak over the critics' 333,826 parameters with their targets
    and the policy's 171,043 without: 18,142,244 bytes), each as `reps`
    back-to-back launches between torch events on the launching stream (so a
    launch's time includes its share of the launch boundaries)."""
    from oac_amd import _lib
    L = _lib.lib()
    sp = _lib.stream_ptr()
    rs = np.random.RandomState(5)
    idx = torch.from_numpy(rs.randint(0, rb._storage.shape[0], B).astype(np.int32)).to(device)
    out = torch.empty(B, rb._storage.shape[1], device=device)

    def ev_time(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) * 1e3 / reps   # us per call

    p = lambda t: ctypes.c_void_p(t.data_ptr())
    us_g = ev_time(lambda: _lib.check(L.oac_replay_gather(p(rb._storage), rb._storage.shape[1], p(idx),
                                                          B, p(out), sp)))
    # the arenas' 16-byte padding: 333,828 / 171,044 floats (the bytes below
    # stay SURVEY 8d's unpadded count)
    nq, npol = 333_828, 171_044
    bufs = [torch.zeros(n, device=device) for n in (nq, nq, nq, nq, nq, npol, npol, npol, npol)]
    state = torch.zeros(16, dtype=torch.int64, device=device)
    qp, qg, qm, qv, qt, pp_, pg, pm, pv = bufs

    def adam():
        _lib.check(L.oac_adam_polyak(p(qp), p(qg), p(qm), p(qv), nq, p(qt), 5e-3, 1, 3e-4, 0.9, 0.999,
                                     1e-8, p(state), 0, sp))
        _lib.check(L.oac_adam_polyak(p(pp_), p(pg), p(pm), p(pv), npol, None, 5e-3, 1, 3e-4, 0.9, 0.999,
                                     1e-8, p(state), 1, sp))
    us_a = ev_time(adam)
    gbytes = (GATHER_BYTES_PER_SAMPLE + 3_081) * B
    return {"gather": {"B": B, "bytes": gbytes, "us": round(us_g, 3),
                       "GBps": round(gbytes / us_g / 1e3, 1),
                       "frac_of_hbm_peak": round(gbytes / us_g / 1e3 / PEAK_HBM_GBS, 4)},
            "adam_polyak": {"bytes": ADAM_BYTES_PER_STEP, "us": round(us_a, 3), "launches": 2,
                            "GBps": round(ADAM_BYTES_PER_STEP / us_a / 1e3, 1),
                            "frac_of_hbm_peak": round(ADAM_BYTES_PER_STEP / us_a / 1e3 / PEAK_HBM_GBS, 4)},
            "method": "%d back-to-back launches between torch events on the launching stream" % reps}


def batch_leg(name, tr, rb, B, steps, warmup, flop_per_sample, world, device, timing_steps=8,
              rank=0, seed=101, traffic_key=None, exec_flop_per_sample=None):
    """The drop-in loop at another batch size on the same trainer (every rank
    steps: at world > 1 this is the data-parallel step), with its own
    kernel timing and roofline."""
    np.random.seed(seed + rank)
    el = timed(dropin_run(tr, rb, B), steps, warmup, world, device)
    kt = kernel_timing(tr, rb, B, timing_steps)
    v = world * steps / el
    out = {"workload": name, "steps_per_s": round(v, 1), "ms_per_step": round(1e3 * el / steps, 4),
           "samples_per_s": round(v * B, 1), "batch_per_rank": B, "steps": steps,
           "step_roofline_frac": round(flop_per_sample * B * v / world / 1e12 / PEAK_FP32_TFLOPS, 4),
           "roofline": roofline_of(kt, flop_per_sample, B, timing_steps, traffic_key,
                                   exec_flop_per_sample),
           "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in d.items()}
                       for k, d in kt.items()}}
    out.update(hbm_legs(kt, B, timing_steps))
    return out


def launch_breakdown(tr, rb, B, n=20, seed=4321):
    """Per-launch device durations (us, median over n drop-in steps) of the
    trainer's step, in issue order, with the kind of each launch (direct
    launches with dispatch events; collectives are not kernels of the plan)."""
    from oac_amd import _lib
    capture = getattr(tr, "capture", None)
    if capture is not None:
        tr.capture = False
    st = np.random.get_state()
    np.random.seed(seed)
    tr.train(rb.random_batch(B))
    plan = tr._last_plan
    L = _lib.lib()
    torch.cuda.synchronize()
    _lib.check(L.oac_sac_set_timing(plan.handle, 1))
    ms = (ctypes.c_double * 4)()
    cnt = (ctypes.c_int64 * 4)()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))   # reset
    for _ in range(n):
        tr.train(rb.random_batch(B))
    torch.cuda.synchronize()
    cap = 64 * n
    t = (ctypes.c_double * cap)()
    k = (ctypes.c_int * cap)()
    m = L.oac_sac_read_launch_times(plan.handle, t, k, cap)
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
    _lib.check(L.oac_sac_set_timing(plan.handle, 0))
    np.random.set_state(st)
    if capture is not None:
        tr.capture = capture
    per = m // n if m > 0 else 0
    if per == 0:
        return {}
    arr = np.array(t[:per * n]).reshape(n, per) * 1e3
    names = ["gemm", "row", "adam", "gather"]
    return {"launches_per_step": per, "sum_us": round(float(np.median(arr, 0).sum()), 2),
            "us": [round(float(x), 2) for x in np.median(arr, 0)],
            "kinds": [names[k[i]] for i in range(per)]}


def dp1_leg(args, rb, device, B, single_value, steps=640, warmup=64):
    """The data-parallel step at ONE rank over RCCL (an in-process process
    group of world size 1): the phase split, the separate critic / policy Adam
    launches and the three all-reduces captured into the step graph, on the
    same drop-in loop and replay as the headline -- what the DP structure
    costs before any link latency."""
    import datetime
    import torch.distributed as dist
    if dist.is_initialized():
        return None
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=device,
                            timeout=datetime.timedelta(seconds=120))
    try:
        import oac_amd
        from oac_amd.dp import DataParallelSACTrainer
        torch.manual_seed(0)
        hid = [args.hidden, args.hidden]
        pp = oac_amd.get_policy_producer(args.obs_dim, args.act_dim, hid, device=device)
        qp = oac_amd.get_q_producer(args.obs_dim, args.act_dim, hid, device=device)
        out = {"batch": B, "steps": steps, "backend": "nccl (RCCL), world_size 1"}
        # (collectives, overlap): the phase split alone; the three all-reduces
        # issued through RCCL although world size is 1; and the schedule an
        # N > 1 run executes -- phases 4 / 5 with the alpha all-reduce on a
        # forked side stream captured into the step graph
        for force, ovl in ((False, False), (True, False), (True, True)):
            with DataParallelSACTrainer(pp, qp, action_space=Space(args.act_dim), discount=0.99,
                                        reward_scale=1.0, policy_lr=3e-4, qf_lr=3e-4,
                                        soft_target_tau=5e-3, target_update_period=1,
                                        use_automatic_entropy_tuning=True, device=device, seed=2,
                                        gemm_cfg=args.gemm_cfg, force_collectives=force,
                                        force_overlap=ovl) as tr:
                np.random.seed(1)
                el = timed(dropin_run(tr, rb, B), steps, warmup, 1, device)
                assert torch.isfinite(tr.params).all().item(), "non-finite DP parameters"
                lb = launch_breakdown(tr, rb, B) if not force else None
            v = steps / el
            leg = {"steps_per_s": round(v, 1), "ms_per_step": round(1e3 * el / steps, 4),
                   "vs_single_process": round(v / single_value, 4)}
            if ovl:
                out["with_rccl_allreduces_overlap_schedule"] = leg
            elif force:
                out["with_rccl_allreduces"] = leg
            else:       # the phase split itself (at world size 1 the sums are identities)
                out.update(leg)
                out["launches"] = lb
        return out
    finally:
        dist.destroy_process_group()


def ring_timing(tr, stream, rb, B, steps=640, n=64):
    """train_from_ring: device MT19937 index ring, n steps per graph launch."""
    step = step_fn(tr, rb, stream, B, n)

    def run(k):
        for _ in range(k // n):
            step()
    el = timed(run, steps, n, 1, None)
    return {"steps_per_s": round(steps / el, 1), "ms_per_step": round(1e3 * el / steps, 4),
            "steps_per_launch": n}


def poac_ant_leg(args, device, B=4096, steps=384, warmup=32, timing_steps=8):
    """BASELINE configs[4]: particle_trainer_oac.ParticleTrainer, K=10 shared
    critic heads, Ant-v2 dims (obs 111, act 8), 2x256, batch 4096, replay 1e6,
    on the drop-in loop."""
    import oac_amd
    from oac_amd import ParticleTrainerOAC, ReplayBuffer
    Do, Da, K = 111, 8, 10
    torch.manual_seed(0)
    pp = oac_amd.get_policy_producer(Do, Da, [256, 256], device=device)
    qp = oac_amd.get_q_producer(Do, Da, [256, 256], output_size=K, device=device)
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), discount=0.99,
                            policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3,
                            use_automatic_entropy_tuning=True, deterministic=False, q_min=0.0,
                            q_max=500.0, share_layers=True, device=device)
    rb = ReplayBuffer(args.replay, Do, Da, device=device)
    rb.load_transitions(synthetic_rows(args.replay, rb.rows, Do, Da, device, seed=3))
    out = batch_leg("particle_trainer_oac K=10, Ant-v2 dims (111, 8), 2x256, batch 4096, "
                    "replay 1e6 (BASELINE configs[4])", tr, rb, B, steps, warmup,
                    FLOP_PER_SAMPLE_POAC_ANT, 1, device, timing_steps, traffic_key="poac4096")
    assert torch.isfinite(tr.params).all().item(), "non-finite P-OAC parameters"
    del tr, rb
    return out


def kernel_timing(tr, rb, B, n, seed=12345):
    """Per-kernel timing of n drop-in steps (direct launches: every launch
    carries a HIP start/stop event pair recorded on its own dispatch,
    hipExtLaunchKernel, so a duration is the kernel's begin->end interval --
    the one rocprofv3's kernel trace reports -- with no event packets or
    launch gaps inside it).  The kernels are the ones the step's graph runs."""
    from oac_amd import _lib
    capture = getattr(tr, "capture", None)
    if capture is not None:
        tr.capture = False   # data-parallel: eager phases while the per-kernel events record
    st = np.random.get_state()
    np.random.seed(seed)

    def step():
        b = rb.random_batch(B)
        tr.train(b)
    step()  # build the plan
    plan = tr._last_plan
    L = _lib.lib()
    torch.cuda.synchronize()
    _lib.check(L.oac_sac_set_timing(plan.handle, 1))
    ms = (ctypes.c_double * 4)()
    cnt = (ctypes.c_int64 * 4)()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))   # reset
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
    _lib.check(L.oac_sac_set_timing(plan.handle, 0))
    np.random.set_state(st)
    if capture is not None:
        tr.capture = capture
    names = ["gemm_grouped", "row", "adam", "gather"]
    return {names[k]: dict(ms=ms[k], launches=int(cnt[k]),
                           avg_us=1e3 * ms[k] / max(cnt[k], 1)) for k in range(4)}


def unpin_host_threads():
    """Every thread of this process back on the cores it started with."""
    if not _HOST_CPUS:
        return
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), _HOST_CPUS)
        except OSError:
            pass


def cpu_threads_all():
    """All cores this process may run on (len(os.sched_getaffinity(0)), capped
    by OMP_NUM_THREADS where the host sets it: the GPU box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(n, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else n), n


def cpu_baseline(args, runs=5, steps=300, warmup=20, all_runs=3, kind="sac", B=None,
                 dims=None):
    """The reference's PyTorch-CPU step restated on torch autograd
    (oracle/sac_autograd.py: the reference's forward ops, backward() and the
    torch-1.4 Adam, pinned against the reference-run goldens in
    tests/test_oracle_golden.py), with the host numpy gather + fp32
    conversion, timed on this host's cores with BASELINE.md section 3's
    procedure, bounded: `warmup` steps, then runs of `steps` steps each -- the
    median of `runs` at 1 thread (the reference launcher's
    torch.set_num_threads(1), launcher_util.py:90) and `all_runs` at all
    cores (none when 0).  kind "sac": SACTrainer (trainer/trainer.py); kind
    "poac": particle_trainer_oac.ParticleTrainer, K=10 shared heads."""
    sys.path.insert(0, ROOT)
    from oracle import sac_oracle as so
    from oracle.sac_autograd import ParticleOACAutograd, SACAutograd
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_lib import sac_params
    Do, Da, H = dims or (args.obs_dim, args.act_dim, args.hidden)
    B = B or args.batch
    n = 100_000
    rs = np.random.RandomState(0)
    data = dict(observations=rs.standard_normal((n, Do)), actions=rs.uniform(-1, 1, (n, Da)),
                rewards=rs.standard_normal((n, 1)),
                terminals=(rs.uniform(0, 1, (n, 1)) < 0.01).astype(np.uint8),
                next_observations=rs.standard_normal((n, Do)))
    rep = so.NumpyReplay(data)
    if kind == "poac":
        K = 10
        orc = ParticleOACAutograd(sac_params(Do, Da, [H, H], 0, q_out=K,
                                             q_last_bias=np.linspace(0.0, 500.0, K)), Do, Da, K)
        what = "P-OAC (particle_trainer_oac K=10) steps"
    else:
        orc = SACAutograd(sac_params(Do, Da, [H, H], 0), Do, Da)
        what = "SAC steps"
    g = torch.Generator().manual_seed(2)
    irs = np.random.RandomState(1)

    def step():
        _, b = rep.random_batch(B, irs)
        e1 = torch.randn(B, Da, generator=g)
        e2 = torch.randn(B, Da, generator=g)
        orc.step(so.NumpyReplay.to_torch(b), e1, e2)

    def median_rate(threads, nruns):
        torch.set_num_threads(threads)
        for _ in range(warmup):
            step()
        rates = []
        for _ in range(nruns):
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            rates.append(steps / (time.perf_counter() - t0))
        return float(np.median(rates)), [round(r, 2) for r in rates]
    one, one_runs = median_rate(1, runs)
    sample = (f"{warmup} warm-up steps, then runs of {steps} {what} of the reference's op "
              f"sequence on torch autograd (oracle/sac_autograd.py; obs {Do}, act {Da}, 2x{H}, "
              f"B={B}, numpy f64 replay of {n} rows, torch CPU fp32)")
    out = dict(value=round(one, 2), unit="grad-steps/s", cores=1, kind="port",
               sample=sample + f", median of {runs} runs, 1 thread", runs=one_runs)
    if all_runs:
        T, aff = cpu_threads_all()
        allc, all_rates = median_rate(T, all_runs)
        out["all_cores"] = dict(value=round(allc, 2), cores=T, affinity_cpus=aff, runs=all_rates,
                                sample=sample + f", median of {all_runs} run(s), {T} threads")
    torch.set_num_threads(1)
    return out


def recipe_cpu_baseline(kind, args, steps=200):
    """The oracle's CPU restatement of the g-oac / p-oac recipe step
    (GaussianOACOracle / ParticleUBOracle, counts=True), same dims / batch,
    on a bounded sample of steps."""
    sys.path.insert(0, ROOT)
    from oracle import sac_oracle as so
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_lib import goac_params, ptrain_params
    torch.set_num_threads(1)
    Do, Da, H, B = args.obs_dim, args.act_dim, args.hidden, args.batch
    n = 20_000
    rs = np.random.RandomState(0)
    data = dict(observations=rs.standard_normal((n, Do)), actions=rs.uniform(-1, 1, (n, Da)),
                rewards=rs.standard_normal((n, 1)),
                terminals=(rs.uniform(0, 1, (n, 1)) < 0.01).astype(np.uint8),
                next_observations=rs.standard_normal((n, Do)))
    rep = so.NumpyReplay(data)
    if kind == "goac":
        orc = so.GaussianOACOracle(goac_params(Do, Da, [H, H], 0, 0.0, 500.0), Do, Da,
                                   q_max=500.0)
    else:
        orc = so.ParticleUBOracle(ptrain_params(Do, Da, [H, H], 0, 10, 0.0, 500.0), Do, Da, 10,
                                  8, q_max=500.0)
    irs = np.random.RandomState(1)
    counts = np.zeros(n)

    def step():
        idx, b = rep.random_batch(B, irs)
        b = so.NumpyReplay.to_torch(b)
        b["counts"] = counts[idx][:, None].copy()
        np.add.at(counts, np.unique(idx), 1)
        orc.step(b)
    for _ in range(20):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return dict(value=round(steps / dt, 2), unit="grad-steps/s", cores=1, kind="port",
                sample=f"20 warm-up steps, then {steps} oracle {kind} steps (Humanoid dims, 2x256, "
                       f"B={B}, counts, torch CPU fp32, 1 thread)")


def exploration_timing(tr, obs_dim, reps=200):
    """get_optimistic_exploration_action latency (one observation, the
    reference's per-env-step call; beta_UB 4.66, delta 23.53) and the
    vectorised throughput at 64 observations per call -- host wall time per
    call including the H2D observation copy and the D2H action copy."""
    from oac_amd import get_optimistic_exploration_action, get_optimistic_exploration_actions
    hp = dict(beta_UB=4.66, delta=23.53, share_layers=False)
    rs = np.random.RandomState(0)
    ob = rs.standard_normal(obs_dim)
    obs64 = rs.standard_normal((64, obs_dim))
    for _ in range(20):
        get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
        get_optimistic_exploration_actions(obs64, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    torch.cuda.synchronize()
    # single-observation latency: median of 5 runs of reps calls (host
    # wall-clock jitter on a shared box moved single runs by ~15 %)
    runs = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(reps):
            get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
        runs.append(1e6 * (time.perf_counter() - t0) / reps)
    t1 = time.perf_counter()
    for _ in range(reps):
        get_optimistic_exploration_actions(obs64, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    t2 = time.perf_counter()
    return {"us_per_call_1obs": round(float(np.median(runs)), 1),
            "us_per_call_1obs_runs": [round(r, 1) for r in runs],
            "actions_per_s_64obs": round(64 * reps / (t2 - t1), 1),
            "beta_UB": 4.66, "delta": 23.53}


def count_replay(args, device):
    """ReplayBufferCount with the same synthetic transitions (the counts=True
    recipes of the g-oac / p-oac legs)."""
    from oac_amd import ReplayBufferCount
    rb = ReplayBufferCount(args.replay, args.obs_dim, args.act_dim, device=device)
    rb.load_transitions(synthetic_rows(args.replay, rb.rows, args.obs_dim, args.act_dim,
                                       device, seed=0))
    return rb


def recipe_timing(kind, args, device, rb, steps=640, warmup=64, n=64):
    """SURVEY 8f row 3 trainers in their Humanoid recipe configuration, on the
    same replay and dims, gradient steps/s from the device index ring (n steps
    per graph launch; counts read and bumped inside the step):
      goac: GaussianTrainer, reproduce_g-oac.sh (--share_layers --counts,
            deterministic policy, r_max 5 -> q_max 500);
      poac: particle_trainer.ParticleTrainer, reproduce_p-oac_humanoid_counts.sh
            (--n_estimators 10 --share_layers --counts, deterministic policy)."""
    import oac_amd
    from oac_amd import DeviceIndexStream, GaussianTrainer, ParticleTrainer
    torch.manual_seed(0)
    hid = [args.hidden, args.hidden]
    K = 2 if kind == "goac" else 10
    pp = oac_amd.get_policy_producer(args.obs_dim, args.act_dim, hid, device=device)
    qp = oac_amd.get_q_producer(args.obs_dim, args.act_dim, hid, output_size=K, device=device)
    kw = dict(action_space=Space(args.act_dim), discount=0.99, policy_lr=3e-4, qf_lr=3e-4,
              soft_target_tau=5e-3, q_min=0.0, q_max=500.0, share_layers=True, counts=True,
              device=device, gemm_cfg=args.gemm_cfg)
    tr = GaussianTrainer(pp, qp, **kw) if kind == "goac" else \
        ParticleTrainer(pp, qp, n_estimators=K, delta=0.95, **kw)
    stream = DeviceIndexStream(rb, args.batch, chunk=64, seed=11)
    cs = rb.device_count_state()

    def step():
        stream.before_step(n)
        tr.train_from_ring(rb._storage, stream.ring, stream.slots, args.batch, n_steps=n,
                           count_state=cs)
    for _ in range(warmup // n):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // n):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert torch.isfinite(tr.params).all().item(), f"non-finite {kind} parameters"
    return {"steps_per_s": round(steps / el, 1), "ms_per_step": round(1e3 * el / steps, 4),
            "batch": args.batch, "K": K, "counts": True, "steps": steps, "steps_per_launch": n,
            "launches_per_step": int(_launches(tr))}


def _launches(tr):
    from oac_amd import _lib
    return _lib.lib().oac_sac_launch_count(tr._last_plan.handle)


def rocprof_gemm_avg(key, round_dir="r06"):
    """(average GEMM launch us, path) from the committed rocprofv3 summary of
    this workload (tools/prof_summary.py output), or None."""
    for rd in (round_dir, "r05"):   # the newest round's summary, else the previous one
        path = os.path.join("profiles", rd, {256: "b256", 4096: "b4096"}.get(key, str(key))
                            + "_gemm_avg.txt")
        try:
            with open(os.path.join(ROOT, path)) as f:
                for line in f:
                    if line.startswith("GEMM kernel (all instances)"):
                        return float(line.rsplit("avg", 1)[1].split()[0]), path
        except OSError:
            pass
    return None


def load_traffic(B):
    path = os.path.join(ROOT, "profiles", "pmc_gemm_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(str(B))
    except Exception:
        return None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count():
    """GPUs a rank would see, counted without the HIP runtime (the launcher
    process must not initialise the GPU): the KFD topology's GPU nodes (a
    nonzero simd_count), narrowed by ROCR_ / HIP_ / CUDA_VISIBLE_DEVICES.  An
    unreadable topology falls back to torch.cuda.device_count()."""
    import glob
    n = 0
    for path in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(path) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    if n == 0:
        return torch.cuda.device_count()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(n, argv=None):
    """``bench.py --gpus N`` without a launcher: start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment,
    rendezvous on 127.0.0.1) and return the worst exit code.  The parent makes
    no HIP call (the device count comes from the KFD topology), so the ranks
    start on a clean device; a rank that fails takes the others down."""
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    pending = set(range(n))
    while pending:
        for r in list(pending):
            code = procs[r].poll()
            if code is None:
                continue
            pending.discard(r)
            if code != 0:
                rc = rc or code
                for q in pending:   # one rank down: the collectives of the others would hang
                    procs[q].terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 1


def launcher_selftest(args):
    """--selftest-launcher: the N-rank launch path without a GPU (gloo): every
    rank all-reduces its rank id, rank 0 prints the bench-shaped line."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": "launcher selftest", "n_gpus": world,
                          "rank_sum": float(t.item())}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def cpu_baseline_fresh(args, **kw):
    """cpu_baseline in a fresh, unpinned process: its thread pools (torch's,
    the BLAS library's) must size themselves on every core this process
    started with, which the pinned timed process's pools may not (its
    all-cores leg measured 78-103 steps/s against 127-131 unpinned on one
    box, tools/r6/cpu_pin_check.sh)."""
    import subprocess
    unpin_host_threads()
    argv = [a for a in sys.argv[1:] if a != "--no-pin"]
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)] + argv +
                       ["--no-pin", "--cpu-baseline-only", json.dumps(kw)],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline process: rc {r.returncode}: {r.stderr[-500:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    args = parse()
    if args.cpu_baseline_only is not None:   # (cpu_baseline_fresh's child: no GPU work)
        print(json.dumps(cpu_baseline(args, **json.loads(args.cpu_baseline_only))), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # started as `python bench.py --gpus N` (no torchrun): become the launcher
        ngpu = visible_gpu_count() if not args.selftest_launcher else args.gpus
        if not args.selftest_launcher and os.environ.get("OAC_BENCH_SAME_DEVICE") != "1" \
                and ngpu < args.gpus:
            print(f"bench.py --gpus {args.gpus}: only {ngpu} GPU(s) visible "
                  "(OAC_BENCH_SAME_DEVICE=1 OAC_BENCH_BACKEND=gloo rehearses N ranks on one GPU)",
                  file=sys.stderr)
            sys.exit(2)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.selftest_launcher:
        launcher_selftest(args)
        return
    # rehearsal of the N-rank path on a 1-GPU box: OAC_BENCH_BACKEND=gloo and
    # OAC_BENCH_SAME_DEVICE=1 put every rank on cuda:0 (RCCL refuses that)
    if os.environ.get("OAC_BENCH_SAME_DEVICE") == "1":
        local = 0
    dp = world > 1 or force_dp()
    if dp:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("OAC_BENCH_BACKEND", "nccl")
        # a finite timeout: a stuck collective ends the rank (non-zero exit)
        # instead of running into the driver's limit
        import datetime
        tmo = datetime.timedelta(seconds=int(os.environ.get("OAC_BENCH_PG_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    B = args.batch
    tr, rb, stream = build(args, rank, world, device)
    n = 1
    if args.mode == "dropin":
        # the reference's own loop, rl_algorithm.py:160-167: per step
        # random_batch(B) (np.random.randint on numpy's global stream, rank r
        # seeded 1 + r) and trainer.train(batch) -- no pre-drawn
        # indices, every draw inside the timed region
        np.random.seed(1 + rank)

        def run(k):
            for _ in range(k):
                train_data = rb.random_batch(B)
                train_data["buffer"] = rb
                tr.train(train_data)
    else:
        # train_from_ring: device MT19937 index ring, n steps per graph launch
        # (the largest n <= --steps-per-launch dividing the ring chunk, K and W)
        n = max(1, args.steps_per_launch)
        if dp:
            n = min(n, 8)   # data parallel: at most 8 steps (24 RCCL all-reduces) per graph
        while n > 1 and (stream.chunk % n or args.steps % n or args.warmup % n):
            n -= 1
        step = step_fn(tr, rb, stream, B, n)

        def run(k):
            for _ in range(k // n):
                step()

    def barrier():
        torch.cuda.synchronize()
        if dp:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    # no Python garbage collection inside the timed region: a 20-step window
    # is ~2 ms, and a collection pause is a visible share of it.  The collection
    # runs before the warm-up, which then re-warms the host caches it walked
    # (collected right before the window, the first step's host work took
    # 200-350 us instead of ~50: tools/fill_drain.py, round 5)
    gc.collect()
    gc.disable()
    try:
        run(args.warmup)
        barrier()
        t0 = time.perf_counter()
        run(args.steps)
        barrier()
        elapsed = time.perf_counter() - t0
    finally:
        gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = world * args.steps / elapsed
    # sanity: the trained state is finite
    assert torch.isfinite(tr.params).all().item(), "non-finite parameters"

    kt = kernel_timing(tr, rb, B, args.timing_steps)   # every rank steps (collectives)
    # configs[2] (N = 1) / configs[3] (N > 1): the same trainer at batch 4096 per rank
    big = None
    if not args.no_extras and B != 4096:
        big = batch_leg("SAC/OAC trainer step, Humanoid-v2 dims, 2x256, batch 4096 per rank, "
                        "replay 1e6 (BASELINE configs[%d])" % (3 if world > 1 else 2),
                        tr, rb, 4096, 320, 32, FLOP_PER_SAMPLE, world, device, rank=rank,
                        exec_flop_per_sample=EXEC_FLOP_PER_SAMPLE)
    out = None
    if rank == 0:
        roof = roofline_of(kt, FLOP_PER_SAMPLE, B, args.timing_steps,
                           exec_flop_per_sample=EXEC_FLOP_PER_SAMPLE)
        # B >= 1024: per-launch choice among gemm_fwd_kernel (forward),
        # gemm_bwdp_kernel (backward) and gemm_small_kernel (narrow products)
        roof["kernel"] = ("gemm_small_kernel" if B < 1024 else
                          "gemm launches (gemm_fwd / gemm_bwdp / gemm_small)")
        out = {
            "metric": "OAC gradient steps/sec, Humanoid-v2 dims, batch 256, 1->8 MI355X",
            "value": round(value, 2),
            "unit": "grad-steps/s (batch %d per rank)" % B,
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (random-init weights, synthetic transitions)",
            "config": {"workload": "SAC/OAC trainer step, Humanoid-v2 dims (obs 376, act 17), "
                                   "2x256 MLP, replay 1e6 (BASELINE configs[1])",
                       "obs_dim": args.obs_dim, "act_dim": args.act_dim,
                       "hidden": args.hidden, "batch_per_rank": B, "global_batch": B * world,
                       "replay_per_rank": args.replay,
                       "parallelism": "dp%d" % world if dp else "single",
                       "loop": ("rl_algorithm.py:160-167: random_batch(B) + train(batch) per step"
                                if args.mode == "dropin" else
                                "train_from_ring, %d steps per graph launch" % n)},
            "samples_per_s": round(value * B, 1),
            "mode": args.mode,
            "roofline": roof,
            "step_roofline_frac": round(FLOP_PER_SAMPLE * B * value / world / 1e12
                                        / PEAK_FP32_TFLOPS, 5),
            "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv
                            for kk, vv in v.items()} for k, v in kt.items()},
        }
        if big is not None:
            out["b4096"] = big
        out.update(hbm_legs(kt, B, args.timing_steps))
        if world == 1 and not args.no_extras:
            out["launches"] = launch_breakdown(tr, rb, B)
            out["hbm_subkernels"] = standalone_hbm(rb, device)
            # (the device-ring path, train_from_ring, is no longer a default
            # leg: in the drop-in step's form it runs ~8 % below the drop-in
            # loop -- 11,100 against 12,000 steps/s on one box, round 6,
            # tools/r6/ring_ab.sh; `--mode ring` times it)
            if args.mode == "dropin":
                if not dp:
                    try:
                        out["dp1"] = dp1_leg(args, rb, device, B, value)
                    except Exception as e:   # the headline stands without this leg
                        out["dp1"] = {"error": repr(e)[:300]}
            out["exploration"] = exploration_timing(tr, args.obs_dim)
            out["poac_ant_b4096"] = poac_ant_leg(args, device)
            rbc = count_replay(args, device)
            for kind in ("goac", "poac"):
                out[kind] = recipe_timing(kind, args, device, rbc)
                if not args.no_cpu_baseline:
                    out[kind]["cpu_baseline"] = recipe_cpu_baseline(kind, args)
        if not args.no_cpu_baseline and world == 1:   # the CPU baseline is an N=1 figure
            out["cpu_baseline"] = cpu_baseline_fresh(args)
            if big is not None:      # configs[2]: the same step at batch 4096
                # runs of >= 2 s: ~5 steps/s at one thread
                out["b4096"]["cpu_baseline"] = cpu_baseline_fresh(args, steps=11, warmup=2, all_runs=0,
                                                                  B=4096)
            if "poac_ant_b4096" in out:   # configs[4]: P-OAC K=10, Ant dims, batch 4096
                out["poac_ant_b4096"]["cpu_baseline"] = cpu_baseline_fresh(   # (~12.7 steps/s: >= 2 s runs)
                    args, steps=26, warmup=2, all_runs=0, kind="poac", B=4096, dims=[111, 8, 256])
        print(json.dumps(out), flush=True)
    if dp:
        # the trainer's teardown (its captured step graphs hold RCCL kernels),
        # then the process group
        tr.close()
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
