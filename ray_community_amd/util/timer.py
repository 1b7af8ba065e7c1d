"""Lightweight timing helper (reference: ``python/ray/util/timer.py``)."""
from __future__ import annotations

import time


class _Timer:
    def __init__(self, window_size: int = 10):
        self._window = window_size
        self._samples = []
        self._units = []
        self._t0 = None
        self.count = 0

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.push(time.perf_counter() - self._t0)

    def push(self, dt: float):
        self._samples.append(dt)
        self._samples = self._samples[-self._window:]
        self.count += 1

    def push_units_processed(self, n):
        self._units.append(n)
        self._units = self._units[-self._window:]

    def has_units_processed(self):
        return bool(self._units)

    @property
    def mean(self):
        return sum(self._samples) / len(self._samples) if self._samples else 0.0

    @property
    def mean_units_processed(self):
        return sum(self._units) / len(self._units) if self._units else 0.0

    @property
    def mean_throughput(self):
        t = sum(self._samples)
        return sum(self._units) / t if t > 0 else 0.0
