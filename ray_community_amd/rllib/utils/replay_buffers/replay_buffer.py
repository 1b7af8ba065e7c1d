"""Replay buffers (reference: ``rllib/utils/replay_buffers``): uniform ring buffer and
proportional prioritized replay (sum-tree)."""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ...policy.sample_batch import SampleBatch


class ReplayBuffer:
    def __init__(self, capacity: int = 50000, seed: Optional[int] = None):
        self.capacity = int(capacity)
        self.storage: Dict[str, np.ndarray] = {}
        self.size = 0
        self.idx = 0
        self.rng = np.random.default_rng(seed)
        self.num_added = 0

    def __len__(self):
        return self.size

    def add(self, batch: SampleBatch):
        n = batch.count
        if not self.storage:
            for k, v in batch.items():
                self.storage[k] = np.empty((self.capacity,) + v.shape[1:], dtype=v.dtype)
        pos = (self.idx + np.arange(n)) % self.capacity
        for k, v in batch.items():
            self.storage[k][pos] = v
        self.idx = (self.idx + n) % self.capacity
        self.size = min(self.capacity, self.size + n)
        self.num_added += n
        return pos

    def sample(self, num_items: int, **kw) -> SampleBatch:
        idx = self.rng.integers(0, self.size, num_items)
        b = SampleBatch({k: v[idx] for k, v in self.storage.items()})
        b["batch_indexes"] = idx
        return b

    def stats(self, debug: bool = False) -> dict:
        out = {"added_count": self.num_added, "num_entries": self.size, "capacity": self.capacity,
               "est_size_bytes": int(sum(v.nbytes for v in self.storage.values()))}
        if debug:
            out["write_index"] = self.idx
        return out

    def get_state(self):
        return {"storage": self.storage, "size": self.size, "idx": self.idx}

    def set_state(self, st):
        self.storage, self.size, self.idx = st["storage"], st["size"], st["idx"]


class PrioritizedReplayBuffer(ReplayBuffer):
    def __init__(self, capacity=50000, alpha=0.6, seed=None):
        super().__init__(capacity, seed)
        self.alpha = alpha
        self.tree_cap = 1
        while self.tree_cap < self.capacity:
            self.tree_cap *= 2
        self.sum = np.zeros(2 * self.tree_cap)
        self.max_p = 1.0

    def _set(self, idx, p):
        i = idx + self.tree_cap
        self.sum[i] = p
        i //= 2
        while np.any(i >= 1):
            self.sum[i] = self.sum[2 * i] + self.sum[2 * i + 1]
            i //= 2
            if np.all(i == 0):
                break

    def add(self, batch):
        pos = super().add(batch)
        for p in pos:
            self._set(np.array([p]), self.max_p ** self.alpha)
        return pos

    def sample(self, num_items, beta=0.4, **kw):
        total = self.sum[1]
        us = self.rng.uniform(0, total, num_items)
        idx = np.empty(num_items, dtype=np.int64)
        for j, u in enumerate(us):
            i = 1
            while i < self.tree_cap:
                if u <= self.sum[2 * i]:
                    i = 2 * i
                else:
                    u -= self.sum[2 * i]
                    i = 2 * i + 1
            idx[j] = min(i - self.tree_cap, self.size - 1)
        p = self.sum[idx + self.tree_cap] / total
        w = (self.size * np.maximum(p, 1e-12)) ** (-beta)
        b = SampleBatch({k: v[idx] for k, v in self.storage.items()})
        b["weights"] = (w / w.max()).astype(np.float32)
        b["batch_indexes"] = idx
        return b

    def update_priorities(self, idx, prios):
        for i, p in zip(idx, prios):
            self.max_p = max(self.max_p, float(p))
            self._set(np.array([i]), float(p) ** self.alpha)
