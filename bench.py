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
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))

FLOP_PER_SAMPLE = 4_377_600        # algorithmic GEMM FLOPs per sample (SAC, Humanoid)
GATHER_BYTES_PER_SAMPLE = 3_081 + 4
ADAM_BYTES_PER_STEP = 18_142_244
PEAK_FP32_TFLOPS = 157.3           # MI355X fp32 MFMA dense peak (MI355X_MICROARCH.md)
LAUNCH_FLOOR_US = 5.2      # grouped-GEMM launch floor in a graph chain (tools/micro, r01)
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
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the exploration and g-oac legs (profiling runs: keeps the "
                         "per-kernel statistics to the headline step)")
    ap.add_argument("--cpu-steps", type=int, default=1200)
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--timing-steps", type=int, default=50)
    ap.add_argument("--gemm-cfg", type=int, default=-1)
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
    from oac_amd import DeviceIndexStream, ReplayBufferCount, SACTrainer
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
    # ReplayBufferCount (per-row counts for the counts=True recipe legs; the
    # SAC step ignores them)
    rb = ReplayBufferCount(args.replay, args.obs_dim, args.act_dim, device=device)
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


def kernel_timing(tr, rb, stream, B, n):
    """Per-kernel timing of n steps (direct launches on the trainer's stream):
    every launch carries a HIP start/stop event pair recorded on its own
    dispatch (hipExtLaunchKernel), so a duration is the kernel's begin->end
    interval -- the one rocprofv3's kernel trace reports -- with no event
    packets or launch gaps inside it."""
    from oac_amd import _lib
    step = step_fn(tr, rb, stream, B)
    if hasattr(tr, "capture"):
        tr.capture = False   # data-parallel: eager phases while the per-kernel events record
    step()  # build the plan
    plan = tr._last_plan
    L = _lib.lib()
    _lib.check(L.oac_sac_set_timing(plan.handle, 1))
    ms = (ctypes.c_double * 4)()
    cnt = (ctypes.c_int64 * 4)()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))   # reset
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    _lib.check(L.oac_sac_read_timing(plan.handle, ms, cnt, 4))
    _lib.check(L.oac_sac_set_timing(plan.handle, 0))
    names = ["gemm_grouped", "row", "adam", "gather"]
    return {names[k]: dict(ms=ms[k], launches=int(cnt[k]),
                           avg_us=1e3 * ms[k] / max(cnt[k], 1)) for k in range(4)}


def cpu_baseline(args):
    """The oracle's PyTorch-CPU restatement of the reference step (incl. the
    host numpy gather + fp32 conversion), timed on this host's cores."""
    sys.path.insert(0, ROOT)
    from oracle import sac_oracle as so
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_lib import sac_params
    torch.set_num_threads(args.cpu_threads)
    Do, Da, H, B = args.obs_dim, args.act_dim, args.hidden, args.batch
    n = 100_000
    rs = np.random.RandomState(0)
    data = dict(observations=rs.standard_normal((n, Do)), actions=rs.uniform(-1, 1, (n, Da)),
                rewards=rs.standard_normal((n, 1)),
                terminals=(rs.uniform(0, 1, (n, 1)) < 0.01).astype(np.uint8),
                next_observations=rs.standard_normal((n, Do)))
    rep = so.NumpyReplay(data)
    orc = so.SACOracle(sac_params(Do, Da, [H, H], 0), Do, Da)
    g = torch.Generator().manual_seed(2)
    irs = np.random.RandomState(1)

    def step():
        _, b = rep.random_batch(B, irs)
        e1 = torch.randn(B, Da, generator=g)
        e2 = torch.randn(B, Da, generator=g)
        orc.step(so.NumpyReplay.to_torch(b), e1, e2)
    for _ in range(5):
        step()
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        step()
    dt = time.perf_counter() - t0
    return dict(value=args.cpu_steps / dt, unit="grad-steps/s", cores=args.cpu_threads,
                kind="port",
                sample=f"{args.cpu_steps} oracle SAC steps (Humanoid dims, 2x256, B={B}, "
                       f"numpy f64 replay of {n} rows, torch CPU fp32, "
                       f"{args.cpu_threads} thread(s))")


def recipe_cpu_baseline(kind, args, steps=200):
    """The oracle's CPU restatement of the g-oac / p-oac recipe step
    (GaussianOACOracle / ParticleUBOracle, counts=True), same dims / batch,
    on a bounded sample of steps."""
    sys.path.insert(0, ROOT)
    from oracle import sac_oracle as so
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from fixtures_lib import goac_params, ptrain_params
    torch.set_num_threads(args.cpu_threads)
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
    for _ in range(3):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return dict(value=round(steps / dt, 2), unit="grad-steps/s", cores=args.cpu_threads,
                kind="port",
                sample=f"{steps} oracle {kind} steps (Humanoid dims, 2x256, B={B}, counts, "
                       f"torch CPU fp32, {args.cpu_threads} thread(s))")


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
    t0 = time.perf_counter()
    for _ in range(reps):
        get_optimistic_exploration_action(ob, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    t1 = time.perf_counter()
    for _ in range(reps):
        get_optimistic_exploration_actions(obs64, policy=tr.policy, qfs=tr.qfs, hyper_params=hp)
    t2 = time.perf_counter()
    return {"us_per_call_1obs": round(1e6 * (t1 - t0) / reps, 1),
            "actions_per_s_64obs": round(64 * reps / (t2 - t1), 1),
            "beta_UB": 4.66, "delta": 23.53}


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


def load_traffic(B):
    path = os.path.join(ROOT, "profiles", "pmc_gemm_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(str(B))
    except Exception:
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank path on a 1-GPU box: OAC_BENCH_BACKEND=gloo and
    # OAC_BENCH_SAME_DEVICE=1 put every rank on cuda:0 (RCCL refuses that)
    if os.environ.get("OAC_BENCH_SAME_DEVICE") == "1":
        local = 0
    dp = world > 1 or force_dp()
    if dp:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("OAC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    B = args.batch
    tr, rb, stream = build(args, rank, world, device)
    # n steps per graph replay (data-parallel: the phases and RCCL all-reduces
    # of n steps captured together, oac_amd/dp.py)
    # (the largest n <= --steps-per-launch dividing the ring chunk, K and W, so
    # any --steps / --warmup work; the defaults keep n = 64)
    n = max(1, args.steps_per_launch)
    if dp:
        n = min(n, 8)   # data parallel: at most 8 steps (24 RCCL all-reduces) per captured graph
    while n > 1 and (stream.chunk % n or args.steps % n or args.warmup % n):
        n -= 1
    step = step_fn(tr, rb, stream, B, n)

    def barrier():
        torch.cuda.synchronize()
        if dp:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup // n):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps // n):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = world * args.steps / elapsed
    # sanity: the trained state is finite
    assert torch.isfinite(tr.params).all().item(), "non-finite parameters"

    kt = kernel_timing(tr, rb, stream, B, args.timing_steps)   # every rank steps (collectives)
    out = None
    if rank == 0:
        gk = kt["gemm_grouped"]
        flops_per_launch = FLOP_PER_SAMPLE * B * args.timing_steps / max(gk["launches"], 1)
        achieved = flops_per_launch / (gk["avg_us"] * 1e-6) / 1e12
        traffic = load_traffic(B)
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
                       "parallelism": "dp%d" % world if dp else "single"},
            "samples_per_s": round(value * B, 1),
            "steps_per_launch": n,
            "roofline": {"bound": "mfma",
                         # B >= 1024: per-launch choice among gemm_big_kernel (forward),
                         # gemm_grouped_kernel (backward) and gemm_small_kernel (narrow)
                         "kernel": "gemm_small_kernel" if B < 1024 else
                                   "gemm launches (gemm_big/gemm_grouped/gemm_small)",
                         "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         "traffic": traffic,
                         "flops_per_launch": round(flops_per_launch),
                         "avg_launch_us": round(gk["avg_us"], 3)},
            "step_roofline_frac": round(FLOP_PER_SAMPLE * B * value / world / 1e12
                                        / PEAK_FP32_TFLOPS, 5),
            # the bound that actually applies at B=256: a dependent chain of
            # launches, each costing at least the measured floor of a grouped
            # GEMM launch in a hipGraph chain (tools/micro/floor_micro.hip:
            # 5.2 us for 256 tiles of 32x32, K=256)
            "latency_floor": {"launches_per_step": int(_launches(tr)),
                              "floor_us_per_launch": LAUNCH_FLOOR_US,
                              "floor_us_per_step": round(LAUNCH_FLOOR_US * _launches(tr), 2),
                              "frac": round(LAUNCH_FLOOR_US * _launches(tr)
                                            / (1e3 * ms_per_step), 4)},
            "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv
                            for kk, vv in v.items()} for k, v in kt.items()},
        }
        ga, ad = kt["gather"], kt["adam"]
        if ga["launches"]:
            out["gather_GBps"] = round(GATHER_BYTES_PER_SAMPLE * B / (ga["avg_us"] * 1e-6) / 1e9, 1)
        if ad["launches"]:
            out["adam_GBps"] = round(ADAM_BYTES_PER_STEP * args.timing_steps / (ad["ms"] * 1e-3) / 1e9, 1)
        if world == 1 and not args.no_extras:
            out["exploration"] = exploration_timing(tr, args.obs_dim)
            for kind in ("goac", "poac"):
                out[kind] = recipe_timing(kind, args, device, rb)
                if not args.no_cpu_baseline:
                    out[kind]["cpu_baseline"] = recipe_cpu_baseline(kind, args)
        if not args.no_cpu_baseline and world == 1:   # the CPU baseline is an N=1 figure
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if dp:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
