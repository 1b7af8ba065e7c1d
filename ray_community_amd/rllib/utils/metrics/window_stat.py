"""A fixed-window running statistic (reference: rllib/utils/metrics/window_stat.py)."""
from __future__ import annotations

import collections

import numpy as np


class WindowStat:
    def __init__(self, name: str, n: int):
        self.name = name
        self.items = collections.deque(maxlen=int(n))
        self.count = 0

    def push(self, obj) -> None:
        self.items.append(obj)
        self.count += 1

    def mean(self) -> float:
        return float(np.mean(self.items)) if self.items else float("nan")

    def std(self) -> float:
        return float(np.std(self.items)) if self.items else float("nan")

    def quantiles(self):
        return np.percentile(self.items, [0, 10, 50, 90, 100]).tolist() if self.items else []

    def stats(self) -> dict:
        return {self.name + "_count": int(self.count), self.name + "_mean": self.mean(),
                self.name + "_std": self.std(), self.name + "_quantiles": self.quantiles()}
