"""ReplayBuffer insert path and ReplayBufferCount (replay_buffer.py:50-104,
151-197) against golden runs of the reference's own ReplayBufferCount
(tests/golden/make_golden.py gen_replay_count): the CPU restatement
(oracle/replay_oracle.py) on the CPU, the device buffer (HIP insert kernel,
counts bookkeeping, priority sampling) on the GPU.

Bars: drawn indices, batch counts and the counts array exact; stored rows
equal to the reference's float64 fields rounded to fp32 (bit-exact)."""
import numpy as np
import pytest

import parity

CASES = ["replay_count", "replay_count_priority"]


def _ops(meta, g):
    for k in range(len(meta["path_lengths"])):
        path = {key: g[f"op{k}/path/{key}"] for key in
                ("observations", "actions", "rewards", "next_observations", "terminals")}
        path["agent_infos"] = [{}] * len(path["observations"])
        path["env_infos"] = [{}] * len(path["observations"])
        yield k, path


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_golden(name):
    from oracle.replay_oracle import CountReplayOracle
    meta, g = parity.load(name)
    o = CountReplayOracle(meta["N"], meta["obs_dim"], meta["act_dim"], meta["priority"])
    np.random.seed(meta["np_seed"])
    for k, path in _ops(meta, g):
        o.add_path(path)
        batch, idx, u = o.random_batch(meta["B"])
        np.testing.assert_array_equal(batch["observations"], g[f"op{k}/obs"])
        np.testing.assert_array_equal(batch["counts"][:, 0], g[f"op{k}/counts_batch"])
        np.testing.assert_array_equal(o.counts[:, 0], g[f"op{k}/counts_after"])
        if meta["priority"]:
            np.testing.assert_array_equal(u, g[f"op{k}/u"])
    np.testing.assert_array_equal(o.obs, g["final/observations"])
    np.testing.assert_array_equal([o.top, o.size], g["final/top_size"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_device_count_buffer_matches_reference_golden(name):
    import torch
    from gpu_helpers import Space
    from oac_amd import ReplayBufferCount
    meta, g = parity.load(name)
    rb = ReplayBufferCount(meta["N"], Space(meta["obs_dim"]), Space(meta["act_dim"]),
                           priority_sample=meta["priority"], device="cuda:0")
    np.random.seed(meta["np_seed"])
    for k, path in _ops(meta, g):
        rb.add_paths([path])
        batch = rb.random_batch(meta["B"])
        obs = batch["observations"].cpu().numpy()
        np.testing.assert_array_equal(obs, g[f"op{k}/obs"].astype(np.float32))
        np.testing.assert_array_equal(batch["counts"].cpu().numpy()[:, 0],
                                      g[f"op{k}/counts_batch"].astype(np.float32))
        np.testing.assert_array_equal(rb._counts.cpu().numpy(), g[f"op{k}/counts_after"])
    torch.cuda.synchronize()
    ss = rb.get_snapshot()
    for key, gk in (("_observations", "final/observations"), ("_actions", "final/actions"),
                    ("_rewards", "final/rewards"), ("_next_obs", "final/next_obs")):
        np.testing.assert_array_equal(ss[key], g[gk].astype(np.float32).astype(np.float64), key)
    np.testing.assert_array_equal(ss["_terminals"], g["final/terminals"])
    np.testing.assert_array_equal([ss["_top"], ss["_size"]], g["final/top_size"])


@pytest.mark.gpu
def test_priority_sampling_follows_inverse_counts():
    """Statistical check at a size the golden run does not reach (200k rows,
    skewed counts): empirical frequencies of 400k priority draws against
    p = 1/(c+1) normalised, per count class (chi-square, 4 classes)."""
    import torch
    from gpu_helpers import Space
    from oac_amd import ReplayBufferCount
    N = 200_000
    rb = ReplayBufferCount(N, Space(3), Space(1), priority_sample=True, device="cuda:0")
    rows = torch.zeros(N, rb.rows["row_stride"], device="cuda:0")
    rb.load_transitions(rows)
    cls = torch.arange(N, device="cuda:0") % 4          # counts 0, 1, 3, 7 by class
    rb._counts.copy_(torch.tensor([0, 1, 3, 7], device="cuda:0", dtype=torch.int32)[cls])
    np.random.seed(0)
    idx = torch.cat([rb._priority_indices(40_000) for _ in range(10)]).long()
    assert int(idx.min()) >= 0 and int(idx.max()) < N
    obs = torch.bincount(cls[idx], minlength=4).cpu().numpy().astype(np.float64)
    w = np.array([1, 1 / 2, 1 / 4, 1 / 8])
    exp = w / w.sum() * obs.sum()
    chi2 = float(((obs - exp) ** 2 / exp).sum())
    assert chi2 < 16.3, (obs, exp, chi2)   # p = 0.001 at 3 dof
