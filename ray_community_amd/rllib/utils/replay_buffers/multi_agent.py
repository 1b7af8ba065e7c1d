"""More replay buffers (reference: rllib/utils/replay_buffers/{fifo,reservoir,multi_agent,
multi_agent_prioritized,multi_agent_mixin,prioritized_episode}_replay_buffer.py).

* ``FifoReplayBuffer``: a queue -- ``sample(n)`` hands out (and drops) the oldest ``n`` items.
* ``ReservoirReplayBuffer``: a uniform sample of everything ever added (reservoir sampling once full).
* ``MultiAgentReplayBuffer`` / ``MultiAgentPrioritizedReplayBuffer``: one underlying buffer per
  policy id; ``add`` takes a ``MultiAgentBatch`` (or a ``SampleBatch`` for the default policy),
  ``sample`` returns a ``MultiAgentBatch``. ``replay_mode=LOCKSTEP`` samples the same indexes for
  every policy (their buffers then hold one row per env step).
* ``MultiAgentMixInReplayBuffer``: every sample mixes the freshly added rows with replayed ones so
  that the replayed share is ``replay_ratio``.
* ``PrioritizedEpisodeReplayBuffer``: an ``EpisodeReplayBuffer`` whose timesteps are drawn with
  probability proportional to priority^alpha, with importance weights and ``update_priorities``.
"""
from __future__ import annotations

from enum import Enum
from typing import Dict, List, Optional

import numpy as np

from ...policy.sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples
from .episode_replay_buffer import EpisodeReplayBuffer
from .replay_buffer import PrioritizedReplayBuffer, ReplayBuffer


class ReplayMode(str, Enum):
    LOCKSTEP = "lockstep"
    INDEPENDENT = "independent"


class StorageUnit(str, Enum):
    TIMESTEPS = "timesteps"
    SEQUENCES = "sequences"
    EPISODES = "episodes"
    FRAGMENTS = "fragments"


class FifoReplayBuffer(ReplayBuffer):
    """First in, first out: each item is handed out once, oldest first."""

    def __init__(self, capacity: int = 10000, seed: Optional[int] = None):
        super().__init__(capacity, seed)
        self._head = 0  # index of the oldest item still queued

    def add(self, batch: SampleBatch):
        n = batch.count
        if n > self.capacity:  # only the newest ``capacity`` rows can be queued
            batch = SampleBatch({k: v[n - self.capacity:] for k, v in batch.items()})
            n = self.capacity
        if self.size + n > self.capacity:  # overflow drops the oldest queued items
            drop = self.size + n - self.capacity
            self._head = (self._head + drop) % self.capacity
            self.size -= drop
        return super().add(batch)

    def sample(self, num_items: int = 1, **kw) -> SampleBatch:
        n = min(int(num_items), self.size)
        idx = (self._head + np.arange(n)) % max(self.capacity, 1)
        out = SampleBatch({k: v[idx] for k, v in self.storage.items()}) if n else SampleBatch({})
        self._head = (self._head + n) % max(self.capacity, 1)
        self.size -= n
        return out


class ReservoirReplayBuffer(ReplayBuffer):
    """Keeps a uniform random subset of all rows ever added (Vitter's algorithm R)."""

    def add(self, batch: SampleBatch):
        rows = batch.count
        if not self.storage:
            for k, v in batch.items():
                self.storage[k] = np.empty((self.capacity,) + v.shape[1:], dtype=v.dtype)
        pos = []
        for i in range(rows):
            self.num_added += 1
            if self.size < self.capacity:
                j = self.size
                self.size += 1
            else:
                j = int(self.rng.integers(0, self.num_added))
                if j >= self.capacity:
                    continue
            for k, v in batch.items():
                self.storage[k][j] = v[i]
            pos.append(j)
        return np.asarray(pos, dtype=np.int64)


def _as_multi(batch) -> MultiAgentBatch:
    if isinstance(batch, MultiAgentBatch):
        return batch
    return MultiAgentBatch({DEFAULT_POLICY_ID: batch}, batch.count)


class MultiAgentReplayBuffer:
    """One replay buffer per policy id (created on first add)."""

    def __init__(self, capacity: int = 10000, *, replay_mode: str = ReplayMode.INDEPENDENT,
                 underlying_buffer_config: Optional[Dict] = None, seed: Optional[int] = None, **kw):
        self.capacity = int(capacity)
        self.replay_mode = ReplayMode(str(getattr(replay_mode, "value", replay_mode)).lower())
        cfg = dict(underlying_buffer_config or {})
        self._buffer_cls = cfg.pop("type", ReplayBuffer)
        self._buffer_kw = cfg
        self._seed = seed
        self.replay_buffers: Dict[str, ReplayBuffer] = {}
        self.rng = np.random.default_rng(seed)

    def _buffer(self, pid) -> ReplayBuffer:
        b = self.replay_buffers.get(pid)
        if b is None:
            b = self.replay_buffers[pid] = self._buffer_cls(self.capacity, seed=self._seed, **self._buffer_kw)
        return b

    def __len__(self):
        return sum(len(b) for b in self.replay_buffers.values())

    def add(self, batch, **kw):
        mb = _as_multi(batch)
        if self.replay_mode == ReplayMode.LOCKSTEP:
            counts = {b.count for b in mb.policy_batches.values()}
            if len(counts) > 1:
                raise ValueError("LOCKSTEP replay needs one row per env step for every policy")
        for pid, b in mb.policy_batches.items():
            self._buffer(pid).add(b)

    def sample(self, num_items: int, policy_id: Optional[str] = None, **kw) -> MultiAgentBatch:
        if policy_id is not None:
            b = self.replay_buffers[policy_id].sample(num_items, **kw)
            return MultiAgentBatch({policy_id: b}, b.count)
        if self.replay_mode == ReplayMode.LOCKSTEP and self.replay_buffers:
            size = min(len(b) for b in self.replay_buffers.values())
            idx = self.rng.integers(0, size, num_items)
            out = {}
            for pid, buf in self.replay_buffers.items():
                sb = SampleBatch({k: v[idx] for k, v in buf.storage.items()})
                sb["batch_indexes"] = idx
                out[pid] = sb
            return MultiAgentBatch(out, num_items)
        out = {pid: buf.sample(num_items, **kw) for pid, buf in self.replay_buffers.items() if len(buf)}
        return MultiAgentBatch(out, num_items)

    def get_state(self) -> Dict:
        return {pid: b.get_state() for pid, b in self.replay_buffers.items()}

    def set_state(self, state: Dict):
        for pid, st in state.items():
            self._buffer(pid).set_state(st)


class MultiAgentPrioritizedReplayBuffer(MultiAgentReplayBuffer):
    def __init__(self, capacity: int = 10000, *, prioritized_replay_alpha: float = 0.6,
                 prioritized_replay_beta: float = 0.4, prioritized_replay_eps: float = 1e-6, **kw):
        cfg = dict(kw.pop("underlying_buffer_config", None) or {})
        cfg.setdefault("type", PrioritizedReplayBuffer)
        cfg.setdefault("alpha", prioritized_replay_alpha)
        super().__init__(capacity, underlying_buffer_config=cfg, **kw)
        self.beta = prioritized_replay_beta
        self.eps = prioritized_replay_eps

    def sample(self, num_items: int, policy_id: Optional[str] = None, beta: Optional[float] = None, **kw):
        return super().sample(num_items, policy_id=policy_id, beta=self.beta if beta is None else beta)

    def update_priorities(self, prio_dict: Dict[str, tuple]):
        """``{policy_id: (batch_indexes, td_errors)}``: new priorities |td| + eps."""
        for pid, (idx, td) in prio_dict.items():
            self.replay_buffers[pid].update_priorities(idx, np.abs(np.asarray(td)) + self.eps)


class MultiAgentMixInReplayBuffer(MultiAgentReplayBuffer):
    """``sample`` returns the rows added since the last sample plus replayed ones, the replayed
    share being ``replay_ratio`` (0: only new data; 1: only replay)."""

    def __init__(self, capacity: int = 10000, *, replay_ratio: float = 0.5, **kw):
        if not 0.0 <= replay_ratio <= 1.0:
            raise ValueError("replay_ratio must be in [0, 1]")
        super().__init__(capacity, **kw)
        self.replay_ratio = replay_ratio
        self._fresh: Dict[str, List[SampleBatch]] = {}

    def add(self, batch, **kw):
        mb = _as_multi(batch)
        for pid, b in mb.policy_batches.items():
            self._fresh.setdefault(pid, []).append(b)
        super().add(mb)

    def sample(self, num_items: Optional[int] = None, policy_id: Optional[str] = None, **kw) -> MultiAgentBatch:
        out = {}
        pids = [policy_id] if policy_id is not None else list(self.replay_buffers)
        for pid in pids:
            fresh = self._fresh.pop(pid, [])
            new = concat_samples(fresh) if fresh else None
            n_new = new.count if new is not None else 0
            if self.replay_ratio >= 1.0:
                n_old = int(num_items or n_new or 1)
                parts = []
            else:
                n_old = int(round(n_new * self.replay_ratio / (1.0 - self.replay_ratio))) if n_new else 0
                parts = [new] if new is not None else []
            if n_old and len(self.replay_buffers[pid]):
                old = self.replay_buffers[pid].sample(n_old)
                old.pop("batch_indexes", None)
                parts.append(old)
            if parts:
                out[pid] = concat_samples(parts)
        return MultiAgentBatch(out, max((b.count for b in out.values()), default=0))


class PrioritizedEpisodeReplayBuffer(EpisodeReplayBuffer):
    def __init__(self, capacity: int = 10000, *, alpha: float = 1.0, beta: float = 0.4, **kw):
        super().__init__(capacity, **kw)
        self.alpha, self.beta = float(alpha), float(beta)
        self._prio: Dict[str, np.ndarray] = {}
        self._max_p = 1.0
        self._last: List[tuple] = []

    def _prios(self):
        live = {e.id_ for e in self.episodes}
        for k in [k for k in self._prio if k not in live]:
            del self._prio[k]
        out = []
        for e in self.episodes:
            a = self._prio.get(e.id_)
            if a is None or len(a) < len(e):
                fill = np.full(len(e) - (0 if a is None else len(a)), self._max_p)
                a = fill if a is None else np.concatenate([a, fill])
                self._prio[e.id_] = a
            out.append(a[:len(e)])
        return out

    def _draw(self, k: int):
        self._num_timesteps_sampled = getattr(self, "_num_timesteps_sampled", 0) + int(k)
        prios = self._prios()
        flat = np.concatenate(prios) ** self.alpha
        p = flat / flat.sum()
        g = self.rng.choice(len(flat), size=k, p=p)
        cum = self._index()
        ei = np.searchsorted(cum, g, side="right")
        ts = g - np.concatenate([[0], cum[:-1]])[ei]
        self._last = [(self.episodes[int(e)].id_, int(t)) for e, t in zip(ei, ts)]
        w = (len(flat) * p[g]) ** (-self.beta)
        self._last_weights = (w / w.max()).astype(np.float32)
        return ei, ts

    def sample(self, num_items: Optional[int] = None, **kw) -> SampleBatch:
        b = super().sample(num_items, **kw)
        if not (kw.get("batch_length_T") or self.batch_length_T):
            b["weights"] = self._last_weights
        return b

    def update_priorities(self, priorities) -> None:
        """New priorities for the timesteps of the last ``sample`` call, in its row order."""
        for (eid, t), p in zip(self._last, np.asarray(priorities, dtype=np.float64)):
            a = self._prio.get(eid)
            if a is not None and t < len(a):
                a[t] = float(p)
                self._max_p = max(self._max_p, float(p))
