"""CPU restatement of the reference replay buffers -- TEST INFRASTRUCTURE ONLY
(the checker for tests/ and nothing else; the product path never imports it).

ReplayBuffer / ReplayBufferCount (/root/reference/replay_buffer.py):
  * ring insert: _top wraps mod capacity, _size saturates (:88-104, :170-178),
    counts of an inserted row reset to 0 (:177);
  * random_batch (:106-115, :180-197): indices by np.random.randint(0, size, B)
    on numpy's global legacy MT19937, or -- priority_sample -- by
    np.random.choice(arange(size), B, p=probs) with probs = 1/(counts+1)
    normalised (:181-184; legacy RandomState.choice with p is
    cdf = cumsum(p), cdf /= cdf[-1], searchsorted(cdf, random_sample(B),
    'right'));  the batch carries counts[indices] BEFORE the update and then
    counts[indices] += 1 -- numpy buffered fancy indexing increments a
    repeated index once.
Pinned by tests/golden/replay_count*.npz, produced by running the reference's
own ReplayBufferCount (tests/golden/make_golden.py, gen_replay_count).
"""
import numpy as np


class CountReplayOracle:
    def __init__(self, capacity, obs_dim, act_dim, priority_sample=False):
        self.N, self.priority = int(capacity), bool(priority_sample)
        self.obs = np.zeros((capacity, obs_dim))
        self.next_obs = np.zeros((capacity, obs_dim))
        self.act = np.zeros((capacity, act_dim))
        self.rew = np.zeros((capacity, 1))
        self.term = np.zeros((capacity, 1), dtype="uint8")
        self.counts = np.zeros((capacity, 1))
        self.top = 0
        self.size = 0

    def add_path(self, path):
        """replay_buffer.py:50-82 + ReplayBufferCount.add_sample (:165-178)."""
        for o, a, r, no, t in zip(path["observations"], path["actions"], path["rewards"],
                                  path["next_observations"], path["terminals"]):
            self.obs[self.top] = o
            self.act[self.top] = a
            self.rew[self.top] = r
            self.term[self.top] = t
            self.next_obs[self.top] = no
            self.counts[self.top] = 0
            self.top = (self.top + 1) % self.N          # _advance, :101-104
            if self.size < self.N:
                self.size += 1

    def indices(self, B, rng=np.random):
        """The draw of random_batch (:180-185) on numpy's global stream."""
        if self.priority:
            probs = 1 / (self.counts[:self.size] + 1)
            probs /= probs.sum()
            p = probs[:, 0]
            cdf = p.cumsum()
            cdf /= cdf[-1]
            u = rng.random_sample(B)
            return cdf.searchsorted(u, side="right"), u
        return rng.randint(0, self.size, B), None

    def random_batch(self, B, rng=np.random):
        idx, u = self.indices(B, rng)
        batch = dict(observations=self.obs[idx], actions=self.act[idx], rewards=self.rew[idx],
                     terminals=self.term[idx], next_observations=self.next_obs[idx],
                     counts=np.copy(self.counts[idx]))
        self.counts[idx] += 1                           # repeated indices: once
        return batch, idx, u
