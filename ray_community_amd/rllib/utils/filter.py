"""Observation filters of the old API stack (reference: rllib/utils/filter.py, filter_manager.py).

``MeanStdFilter`` keeps running mean / variance (Welford) of what it sees; each worker
accumulates a delta ``buffer`` since the last sync, the driver merges the buffers and pushes the
merged filter back (``FilterManager.synchronize``). On the new stack the same job is done by the
``MeanStdFilter`` connector (rllib/connectors/env_to_module.py)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np


class RunningStat:
    def __init__(self, shape=()):
        self.num_pushes = 0
        self.mean_array = np.zeros(shape)
        self.std_array = np.zeros(shape)  # sum of squared deviations (M2)

    def copy(self) -> "RunningStat":
        o = RunningStat(self.mean_array.shape)
        o.num_pushes, o.mean_array, o.std_array = self.num_pushes, self.mean_array.copy(), self.std_array.copy()
        return o

    def push(self, x):
        x = np.asarray(x, dtype=np.float64)
        self.num_pushes += 1
        if self.num_pushes == 1:
            self.mean_array[...] = x
        else:
            delta = x - self.mean_array
            self.mean_array += delta / self.num_pushes
            self.std_array += delta * (x - self.mean_array)

    def update(self, other: "RunningStat"):
        n1, n2 = self.num_pushes, other.num_pushes
        n = n1 + n2
        if n2 == 0:
            return
        delta = other.mean_array - self.mean_array
        self.std_array = self.std_array + other.std_array + delta ** 2 * n1 * n2 / n
        self.mean_array = (n1 * self.mean_array + n2 * other.mean_array) / n
        self.num_pushes = n

    @property
    def n(self):
        return self.num_pushes

    @property
    def mean(self):
        return self.mean_array

    @property
    def var(self):
        return self.std_array / (self.num_pushes - 1) if self.num_pushes > 1 else np.square(self.mean_array)

    @property
    def std(self):
        return np.sqrt(self.var)

    @property
    def shape(self):
        return self.mean_array.shape


class Filter:
    is_concurrent = False

    def apply_changes(self, other: "Filter", *args, **kwargs):
        raise NotImplementedError

    def copy(self) -> "Filter":
        raise NotImplementedError

    def sync(self, other: "Filter"):
        raise NotImplementedError

    def reset_buffer(self):
        raise NotImplementedError

    def as_serializable(self) -> "Filter":
        return self


class NoFilter(Filter):
    def __init__(self, *args):
        pass

    def __call__(self, x, update=True):
        return np.asarray(x)

    def apply_changes(self, other, *args, **kwargs):
        pass

    def copy(self):
        return self

    def sync(self, other):
        pass

    def reset_buffer(self):
        pass


class MeanStdFilter(Filter):
    """``y = (x - mean) / (std + 1e-8)`` (``demean`` / ``destd`` switches), clipped to ±``clip``."""

    def __init__(self, shape, demean: bool = True, destd: bool = True, clip: Optional[float] = 10.0):
        self.shape = shape
        self.demean, self.destd, self.clip = demean, destd, clip
        self.running_stats = RunningStat(shape)
        self.buffer = RunningStat(shape)

    def reset_buffer(self):
        self.buffer = RunningStat(self.shape)

    def apply_changes(self, other: "MeanStdFilter", with_buffer: bool = False, *args, **kwargs):
        """Fold ``other``'s buffered observations into this filter's statistics."""
        self.running_stats.update(other.buffer)
        if with_buffer:
            self.buffer = other.buffer.copy()

    def copy(self) -> "MeanStdFilter":
        o = MeanStdFilter(self.shape, self.demean, self.destd, self.clip)
        o.sync(self)
        return o

    def sync(self, other: "MeanStdFilter"):
        self.demean, self.destd, self.clip = other.demean, other.destd, other.clip
        self.running_stats = other.running_stats.copy()
        self.buffer = other.buffer.copy()

    def __call__(self, x, update: bool = True):
        x = np.asarray(x, dtype=np.float64)
        batched = x.ndim == len(tuple(np.shape(np.zeros(self.shape)))) + 1  # a [B, *shape] batch
        if update:
            rows = x if batched else [x]
            for r in rows:
                self.running_stats.push(r)
                self.buffer.push(r)
        if self.demean:
            x = x - self.running_stats.mean
        if self.destd:
            x = x / (self.running_stats.std + 1e-8)
        if self.clip:
            x = np.clip(x, -self.clip, self.clip)
        return x

    def __repr__(self):
        return f"MeanStdFilter({self.shape}, {self.demean}, {self.destd}, {self.clip}, n={self.running_stats.n})"


class ConcurrentMeanStdFilter(MeanStdFilter):
    is_concurrent = True


def get_filter(filter_config, shape) -> Filter:
    if filter_config == "MeanStdFilter":
        return MeanStdFilter(shape, clip=None)
    if filter_config == "ConcurrentMeanStdFilter":
        return ConcurrentMeanStdFilter(shape, clip=None)
    if filter_config == "NoFilter":
        return NoFilter()
    if callable(filter_config):
        return filter_config(shape)
    raise ValueError(f"Unknown observation_filter: {filter_config!r}")


class FilterManager:
    @staticmethod
    def synchronize(local_filters: Dict[str, Filter], worker_filters: List[Dict[str, Filter]],
                    update_remote: bool = True, timeout_seconds: Optional[float] = None) -> List[Dict[str, Filter]]:
        """Merge each worker's buffered deltas into ``local_filters``; returns the filters every
        worker should ``sync`` to (copies of the merged local ones, buffers cleared)."""
        for wf in worker_filters:
            for k, f in wf.items():
                local_filters[k].apply_changes(f, with_buffer=False)
        merged = {k: f.as_serializable().copy() for k, f in local_filters.items()}
        for f in merged.values():
            f.reset_buffer()
        return [dict(merged) for _ in worker_filters] if update_remote else []


__all__ = ["RunningStat", "Filter", "NoFilter", "MeanStdFilter", "ConcurrentMeanStdFilter", "get_filter",
           "FilterManager"]
