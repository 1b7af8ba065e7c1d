"""Metrics of ``util.iter`` pipelines (reference: python/ray/util/iter_metrics.py): counters,
timers and info dicts shared by the stages of one iterator, merged across shards."""
from __future__ import annotations

import collections
from typing import Dict, List

from .timer import _Timer


class MetricsContext:
    def __init__(self):
        self.counters: Dict[str, int] = collections.defaultdict(int)
        self.timers: Dict[str, _Timer] = collections.defaultdict(_Timer)
        self.info: Dict = {}
        self.current_actor = None

    def save(self):
        return self.counters, self.timers, self.info

    def restore(self, values) -> None:
        self.counters, self.timers, self.info = values


class SharedMetrics:
    """Holds a MetricsContext that several iterators (e.g. a union) read and update."""

    def __init__(self, metrics: MetricsContext = None, parents: List["SharedMetrics"] = None):
        self.metrics = metrics or MetricsContext()
        self.parents = list(parents or [])
        self.set_parents(self.parents)

    def set_parents(self, parents: List["SharedMetrics"]) -> None:
        self.parents = list(parents)
        for p in self.parents:
            p.metrics = self.metrics

    def get(self) -> MetricsContext:
        return self.metrics
