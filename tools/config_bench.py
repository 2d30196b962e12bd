"""Throughput of BASELINE.json configs[4] (particle_trainer_oac K=10 critic,
Ant-v2 dims obs 111 / act 8, batch 4096, replay 1e6, one MI355X) on the
device-ring path -- a parity-test configuration, measured for DESIGN.md.
usage: python tools/config_bench.py [--batch 4096] [--steps 256]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oac-explore_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--replay", type=int, default=1_000_000)
    args = ap.parse_args()
    import oac_amd
    from oac_amd import DeviceIndexStream, ParticleTrainerOAC, ReplayBuffer
    from bench import Space, synthetic_rows
    dev = torch.device("cuda", 0)
    Do, Da, H, K, B = 111, 8, [256, 256], 10, args.batch
    torch.manual_seed(0)
    pp = oac_amd.get_policy_producer(Do, Da, H, device=dev)
    qp = oac_amd.get_q_producer(Do, Da, H, output_size=K, device=dev)
    tr = ParticleTrainerOAC(pp, qp, n_estimators=K, action_space=Space(Da), discount=0.99,
                            policy_lr=3e-4, qf_lr=3e-4, soft_target_tau=5e-3,
                            use_automatic_entropy_tuning=True, deterministic=False, q_min=0.0,
                            q_max=500.0, share_layers=True, device=dev)
    rb = ReplayBuffer(args.replay, Do, Da, device=dev)
    rb.load_transitions(synthetic_rows(args.replay, rb.rows, Do, Da, dev, seed=0))
    st = DeviceIndexStream(rb, B, chunk=64, seed=1)
    n = 64

    def step():
        st.before_step(n)
        tr.train_from_ring(rb._storage, st.ring, st.slots, B, n_steps=n)
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps // n):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert torch.isfinite(tr.params).all().item()
    print(json.dumps({"config": "BASELINE configs[4]: particle_trainer_oac K=10, Ant-v2 dims, "
                                "batch %d, replay %d" % (B, args.replay),
                      "steps_per_s": round(args.steps / el, 1),
                      "ms_per_step": round(1e3 * el / args.steps, 4),
                      "samples_per_s": round(args.steps * B / el, 1)}))


if __name__ == "__main__":
    main()
