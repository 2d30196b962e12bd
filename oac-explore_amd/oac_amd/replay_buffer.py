"""Drop-in ``ReplayBuffer`` (/root/reference/replay_buffer.py:8-148) with the
transitions resident in HBM as fp32 rows.

Row layout (``trainer.row_layout``): ``[obs | act | rew | term | next_obs | pad]``.
Storing fp32 at insert time is bit-identical to the reference's float64 store
converted at sample time (``ptu.from_numpy(...).float()``, utils/core.py:45,
utils/pytorch_util.py:77): rounding f64->f32 is the same operation either way.

``random_batch(B)`` draws the indices exactly like the reference
(``np.random.randint(0, self._size, B)`` on numpy's global legacy MT19937,
replay_buffer.py:107) and returns a ``DeviceBatch``; ``SACTrainer.train``
gathers the rows on the GPU inside the step.  ``index_source='device'``
draws the same stream (np.random.seed(s) semantics) with the device MT19937
kernel instead, so no host work is needed per step.
"""
import ctypes
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr
from .trainer import row_layout

BATCH_KEYS = ("observations", "actions", "rewards", "terminals", "next_observations")


def get_dim(space):
    """utils/env_utils.py:8-18."""
    if isinstance(space, (int, np.integer)):
        return int(space)
    if hasattr(space, "low"):
        return int(np.asarray(space.low).size)
    if hasattr(space, "n"):
        return int(space.n)
    if hasattr(space, "spaces"):
        return sum(get_dim(s) for s in space.spaces)
    if hasattr(space, "flat_dim"):
        return space.flat_dim
    raise TypeError(f"Unknown space: {space}")


class DeviceBatch(dict):
    """The batch dict ``random_batch`` returns: indices on the device plus a
    reference to the HBM store.  Reading a key (e.g. rl_algorithm's
    ``save_sampled_data`` path) gathers that field on the GPU on demand."""

    device_gather = True

    def __init__(self, buffer, indices=None, host_indices=None):
        super().__init__()
        self._buffer, self._indices = buffer, indices
        # host_indices: the np.random.randint draw itself (int64); the trainer
        # stages it through pinned memory inside its step (no pageable copy)
        self.host_indices = host_indices
        self.storage = buffer._storage
        self.batch_size = int(indices.numel() if indices is not None else len(host_indices))

    @property
    def indices(self):
        """The drawn indices as a device int32 tensor (uploaded on first use)."""
        if self._indices is None:
            self._indices = torch.from_numpy(self.host_indices.astype(np.int32)).to(
                self._buffer.device)
        return self._indices

    def __missing__(self, key):
        if key not in BATCH_KEYS:
            raise KeyError(key)
        rows = self._buffer.gather(self.indices)
        r = self._buffer.rows
        spans = dict(observations=(r["off_obs"], self._buffer.ob_dim),
                     actions=(r["off_act"], self._buffer.ac_dim),
                     rewards=(r["off_rew"], 1), terminals=(r["off_term"], 1),
                     next_observations=(r["off_next_obs"], self._buffer.ob_dim))
        o, n = spans[key]
        val = rows[:, o:o + n].contiguous()
        self[key] = val
        return val

    def keys(self):
        return list(BATCH_KEYS) + [k for k in dict.keys(self) if k not in BATCH_KEYS]


class ReplayBuffer(object):
    def __init__(self, max_replay_buffer_size, ob_space, action_space, device=None,
                 index_source="numpy", seed=None):
        self._ob_space, self._action_space = ob_space, action_space
        self.ob_dim, self.ac_dim = get_dim(ob_space), get_dim(action_space)
        self._max_replay_buffer_size = int(max_replay_buffer_size)
        self.rows = row_layout(self.ob_dim, self.ac_dim)
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self._storage = torch.zeros(self._max_replay_buffer_size, self.rows["row_stride"],
                                    dtype=torch.float32, device=self.device)
        self._top = 0
        self._size = 0
        self.index_source = index_source
        self._mt = None
        if index_source == "device":
            self.seed_device_stream(0 if seed is None else seed)

    # ------------------------------------------------------------ insert
    def _rows_from(self, obs, act, rew, nobs, term):
        n = len(obs)
        r = self.rows
        out = np.zeros((n, r["row_stride"]), np.float32)
        out[:, r["off_obs"]:r["off_obs"] + self.ob_dim] = np.asarray(obs).reshape(n, -1)
        out[:, r["off_act"]:r["off_act"] + self.ac_dim] = np.asarray(act).reshape(n, -1)
        out[:, r["off_rew"]] = np.asarray(rew, np.float64).reshape(n)
        out[:, r["off_term"]] = np.asarray(term).reshape(n).astype(np.float32)
        out[:, r["off_next_obs"]:r["off_next_obs"] + self.ob_dim] = np.asarray(nobs).reshape(n, -1)
        return out

    def _write(self, rows_np):
        n = len(rows_np)
        t = torch.from_numpy(rows_np)
        done = 0
        while done < n:
            k = min(n - done, self._max_replay_buffer_size - self._top)
            self._storage[self._top:self._top + k].copy_(t[done:done + k])
            self._top = (self._top + k) % self._max_replay_buffer_size   # _advance, :101-104
            self._size = min(self._size + k, self._max_replay_buffer_size)
            done += k

    def _insert(self, obs, act, rew, nobs, term):
        """Ring insert of n transitions on the device (oac_replay_insert): the
        reference's host dtypes -- float64 fields, uint8 terminals
        (replay_buffer.py:40-45, 92-96) -- are copied once and packed into the
        fp32 rows by a HIP kernel (f64 -> f32 rounding identical to the
        reference's ptu.from_numpy(...).float() at sample time)."""
        n = len(obs)
        if n == 0:
            return
        N = self._max_replay_buffer_size
        top = self._top
        if n > N:   # sequential inserts of n > N rows leave the last N in place
            k = n - N
            top = (top + k) % N
            obs, act, rew, nobs, term = obs[k:], act[k:], rew[k:], nobs[k:], term[k:]
        m = len(obs)

        def dev(x, dt, shape):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(x, dt).reshape(shape))).to(
                self.device)
        o = dev(obs, np.float64, (m, self.ob_dim))
        a = dev(act, np.float64, (m, self.ac_dim))
        r = dev(rew, np.float64, (m,))
        no = dev(nobs, np.float64, (m, self.ob_dim))
        t = dev(np.asarray(term).reshape(m).astype(np.uint8), np.uint8, (m,))
        lay = self.rows
        check(_lib.lib().oac_replay_insert(
            ptr(self._storage), lay["row_stride"], N, top, m, ptr(o), ptr(a), ptr(r), ptr(no),
            ptr(t), self.ob_dim, self.ac_dim, lay["off_obs"], lay["off_act"], lay["off_rew"],
            lay["off_term"], lay["off_next_obs"], stream_ptr()))
        self._on_insert(top, m)
        self._top = (self._top + n) % N                     # _advance, :101-104
        self._size = min(self._size + n, N)

    def _on_insert(self, top, m):
        """Hook: ring positions top .. top+m-1 (mod capacity) were just written."""

    def add_sample(self, observation, action, reward, next_observation, terminal,
                   env_info=None, **kwargs):
        """replay_buffer.py:88-99."""
        if hasattr(self._action_space, "n") and not hasattr(self._action_space, "low"):
            raise AssertionError("discrete action spaces are not supported")
        self._insert([observation], [action], [reward], [next_observation], [terminal])

    def add_path(self, path):
        """replay_buffer.py:50-82: one device insert per path."""
        if len(path["observations"]) == 0:
            return
        self._insert(path["observations"], path["actions"], path["rewards"],
                     path["next_observations"], path["terminals"])

    def add_paths(self, paths):
        for path in paths:
            self.add_path(path)

    def load_transitions(self, rows_fp32):
        """Bulk insert of pre-built device/host rows [n, row_stride] (synthetic fills)."""
        n = rows_fp32.shape[0]
        assert rows_fp32.shape[1] == self.rows["row_stride"] and n <= self._max_replay_buffer_size
        self._storage[:n].copy_(rows_fp32)
        self._top = n % self._max_replay_buffer_size
        self._size = n

    # ------------------------------------------------------------ sample
    def seed_device_stream(self, seed):
        st = np.zeros(625, np.uint32)
        check(_lib.lib().oac_mt_seed_host(ctypes.c_uint32(seed), st.ctypes.data_as(ctypes.c_void_p)))
        self._mt = torch.from_numpy(st.view(np.int32)).to(self.device)

    def sample_indices_device(self, count, out=None):
        """``count`` draws of np.random.randint(0, size) from the device stream."""
        if self._mt is None:
            raise RuntimeError("device index stream not seeded (index_source='device')")
        if out is None:
            out = torch.empty(count, dtype=torch.int32, device=self.device)
        check(_lib.lib().oac_replay_sample_indices(ptr(self._mt), ctypes.c_uint64(self._size),
                                                   int(count), ptr(out), stream_ptr()))
        return out

    def random_batch(self, batch_size):
        """replay_buffer.py:106-115."""
        if self.index_source == "device":
            return DeviceBatch(self, self.sample_indices_device(batch_size))
        return DeviceBatch(self, host_indices=np.random.randint(0, self._size, batch_size))

    def gather(self, indices):
        out = torch.empty(indices.numel(), self.rows["row_stride"], dtype=torch.float32,
                          device=self.device)
        check(_lib.lib().oac_replay_gather(ptr(self._storage), self.rows["row_stride"],
                                           ptr(indices), int(indices.numel()), ptr(out),
                                           stream_ptr()))
        return out

    # ------------------------------------------------------------ misc
    def get_dataset(self):
        r = self.rows
        return self._storage[:self._size, r["off_obs"]:r["off_obs"] + self.ob_dim]

    def num_steps_can_sample(self):
        return self._size

    def get_diagnostics(self):
        return OrderedDict([("size", self._size)])

    def end_epoch(self, epoch):
        return

    def get_snapshot(self):
        """Same keys and dtypes as replay_buffer.py:133-142."""
        r = self.rows
        s = self._storage.cpu().numpy().astype(np.float64)
        return dict(
            _observations=s[:, r["off_obs"]:r["off_obs"] + self.ob_dim],
            _next_obs=s[:, r["off_next_obs"]:r["off_next_obs"] + self.ob_dim],
            _actions=s[:, r["off_act"]:r["off_act"] + self.ac_dim],
            _rewards=s[:, r["off_rew"]:r["off_rew"] + 1],
            _terminals=s[:, r["off_term"]:r["off_term"] + 1].astype(np.uint8),
            _top=self._top, _size=self._size)

    def restore_from_snapshot(self, ss):
        for key in ss.keys():
            assert key in ("_observations", "_next_obs", "_actions", "_rewards", "_terminals",
                           "_top", "_size")
        rows = self._rows_from(ss["_observations"], ss["_actions"], ss["_rewards"],
                               ss["_next_obs"], ss["_terminals"])
        self._storage[:len(rows)].copy_(torch.from_numpy(rows))
        self._top, self._size = int(ss["_top"]), int(ss["_size"])


class ReplayBufferCount(ReplayBuffer):
    """ReplayBufferCount (replay_buffer.py:151-197): per-transition sample
    counts on the device.  random_batch's batch carries ``counts`` (the
    counts of the drawn rows BEFORE this draw, a device float32 [B, 1]; the
    reference returns a float64 copy) and every distinct drawn row's count is
    incremented once (numpy fancy-index ``+=``); ``priority_sample`` draws
    with p = 1/(count+1) (np.random.choice) -- the uniforms are numpy's own
    ``random_sample`` draws on the global stream, exactly the ones the
    reference's choice() consumes, the inverse-cdf search runs on the device
    (oac_replay_priority_sample)."""

    def __init__(self, max_replay_buffer_size, ob_space, action_space, priority_sample=False,
                 device=None, index_source="numpy", seed=None):
        super().__init__(max_replay_buffer_size, ob_space, action_space, device=device,
                         index_source=index_source, seed=seed)
        N = self._max_replay_buffer_size
        self._counts = torch.zeros(N, dtype=torch.int32, device=self.device)
        self._tags = torch.full((N,), -1, dtype=torch.int32, device=self.device)
        self._epoch = 0
        # dedupe epoch of the device ring path (train_from_ring with counts):
        # a device counter, disjoint from the host path's epochs 0, 1, 2, ...
        self._epoch_dev = torch.full((1,), 1 << 30, dtype=torch.int32, device=self.device)
        self.priority_sample = bool(priority_sample)
        self._scratch = None

    def _on_insert(self, top, m):
        """self._counts[self._top] = 0 for every inserted row (:177)."""
        N = self._max_replay_buffer_size
        first = min(m, N - top)
        self._counts[top:top + first].zero_()
        if m > first:
            self._counts[:m - first].zero_()

    def load_transitions(self, rows_fp32):
        super().load_transitions(rows_fp32)
        self._counts.zero_()

    def _priority_indices(self, B):
        L = _lib.lib()
        if self._scratch is None:
            n = int(L.oac_replay_priority_scratch_doubles(self._max_replay_buffer_size))
            self._scratch = torch.empty(n, dtype=torch.float64, device=self.device)
        u = torch.from_numpy(np.random.random_sample(B)).to(self.device)   # choice()'s draws
        idx = torch.empty(B, dtype=torch.int32, device=self.device)
        check(L.oac_replay_priority_sample(ptr(self._counts), self._size, ptr(u), int(B),
                                           ptr(self._scratch), ptr(idx), stream_ptr()))
        return idx

    def random_batch(self, batch_size):
        """replay_buffer.py:180-197."""
        B = int(batch_size)
        if self.priority_sample:
            idx = self._priority_indices(B)
        else:
            idx = super().random_batch(B).indices
        counts = torch.empty(B, dtype=torch.float32, device=self.device)
        check(_lib.lib().oac_replay_counts_update(ptr(self._counts), ptr(self._tags), ptr(idx), B,
                                                  self._epoch, ptr(counts), stream_ptr()))
        self._epoch += 1
        batch = DeviceBatch(self, idx)
        batch["counts"] = counts.view(B, 1)
        return batch

    def device_count_state(self):
        """(counts, tags, epoch) device tensors for trainer.train_from_ring:
        the ring path's steps read / bump these counts like random_batch
        (uniform draws only: priority sampling draws from numpy's stream)."""
        if self.priority_sample:
            raise NotImplementedError("priority_sample draws on the host (np.random.choice); "
                                      "train with random_batch batches")
        return (self._counts, self._tags, self._epoch_dev)

    def get_snapshot(self):
        ss = super().get_snapshot()
        ss["_counts"] = self._counts.cpu().numpy().astype(np.float64).reshape(-1, 1)
        return ss

    def restore_from_snapshot(self, ss):
        ss = dict(ss)
        counts = ss.pop("_counts", None)
        super().restore_from_snapshot(ss)
        if counts is not None:
            self._counts.copy_(torch.from_numpy(np.asarray(counts).reshape(-1).astype(np.int32)))


class DeviceIndexStream:
    """A ring of pre-drawn batch indices for ``SACTrainer.train_from_ring``:
    2*chunk step slots, refilled one chunk ahead by the device MT19937 kernel
    (sequential in the stream, so the index sequence equals
    ``np.random.seed(seed); randint(0, size, B)`` called once per step)."""

    def __init__(self, buffer, batch_size, chunk=64, seed=1):
        self.buf, self.B, self.chunk = buffer, int(batch_size), int(chunk)
        self.slots = 2 * self.chunk
        self.ring = torch.empty(self.slots * self.B, dtype=torch.int32, device=buffer.device)
        buffer.seed_device_stream(seed)
        self.t = 0
        self._fill(0)
        self._fill(1)

    def _fill(self, half):
        view = self.ring[half * self.chunk * self.B:(half + 1) * self.chunk * self.B]
        self.buf.sample_indices_device(self.chunk * self.B, out=view)

    def before_step(self, n_steps=1):
        """Call before each ring step (or block of n_steps consecutive steps,
        n_steps dividing the chunk): refill the half that was just consumed."""
        if self.chunk % n_steps or self.t % n_steps:
            raise ValueError("n_steps must divide the ring chunk and the step count")
        if self.t > 0 and self.t % self.chunk == 0:
            self._fill(((self.t // self.chunk) + 1) % 2)
        self.t += n_steps
