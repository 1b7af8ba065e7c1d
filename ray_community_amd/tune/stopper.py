"""Trial/experiment stoppers (reference: ``python/ray/tune/stopper/``)."""
from __future__ import annotations

import time
from collections import defaultdict, deque
from typing import Callable, Dict, Optional

import numpy as np

from .tuner import Stopper


class NoopStopper(Stopper):
    pass


class FunctionStopper(Stopper):
    def __init__(self, function: Callable[[str, Dict], bool]):
        self._fn = function

    def __call__(self, trial_id, result):
        return bool(self._fn(trial_id, result))

    @classmethod
    def is_valid_function(cls, fn):
        return callable(fn) and not isinstance(fn, Stopper)


class MaximumIterationStopper(Stopper):
    def __init__(self, max_iter: int):
        self._max = max_iter
        self._iter = defaultdict(int)

    def __call__(self, trial_id, result):
        self._iter[trial_id] += 1
        return self._iter[trial_id] >= self._max


class TrialPlateauStopper(Stopper):
    """Stop a trial once the std of its last ``num_results`` metric values is below ``std``."""

    def __init__(self, metric: str, std: float = 0.01, num_results: int = 4, grace_period: int = 4,
                 metric_threshold: Optional[float] = None, mode: Optional[str] = None):
        self._metric, self._std, self._n, self._grace = metric, std, num_results, grace_period
        self._thr, self._mode = metric_threshold, mode
        if metric_threshold is not None and mode not in ("min", "max"):
            raise ValueError("TrialPlateauStopper needs mode='min'|'max' with metric_threshold")
        self._hist = defaultdict(lambda: deque(maxlen=num_results))
        self._count = defaultdict(int)

    def __call__(self, trial_id, result):
        if self._metric not in result:
            return False
        v = float(result[self._metric])
        self._hist[trial_id].append(v)
        self._count[trial_id] += 1
        if self._count[trial_id] < self._grace or len(self._hist[trial_id]) < self._n:
            return False
        if self._thr is not None:
            if self._mode == "max" and v < self._thr:
                return False
            if self._mode == "min" and v > self._thr:
                return False
        return float(np.std(self._hist[trial_id])) <= self._std


class ExperimentPlateauStopper(Stopper):
    """Stop the whole experiment when the best ``top`` results stop improving."""

    def __init__(self, metric: str, std: float = 0.001, top: int = 10, mode: str = "min", patience: int = 0):
        if mode not in ("min", "max"):
            raise ValueError("mode must be 'min' or 'max'")
        self._metric, self._std, self._top, self._mode, self._patience = metric, std, top, mode, patience
        self._results = []
        self._iter = 0
        self._stop = False

    def __call__(self, trial_id, result):
        if self._metric in result:
            self._results.append(float(result[self._metric]))
            self._results.sort(reverse=self._mode == "max")
            self._results = self._results[: self._top]
            if len(self._results) == self._top and float(np.std(self._results)) <= self._std:
                self._iter += 1
            else:
                self._iter = 0
            self._stop = self._iter > self._patience
        return self._stop

    def stop_all(self):
        return self._stop


class TimeoutStopper(Stopper):
    def __init__(self, timeout):
        import datetime

        self._budget = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout)
        self._start = time.time()

    def __call__(self, trial_id, result):
        return False

    def stop_all(self):
        return time.time() - self._start >= self._budget


class CombinedStopper(Stopper):
    def __init__(self, *stoppers: Stopper):
        self._stoppers = stoppers

    def __call__(self, trial_id, result):
        return any([s(trial_id, result) for s in self._stoppers])

    def stop_all(self):
        return any(s.stop_all() for s in self._stoppers)


__all__ = ["Stopper", "NoopStopper", "FunctionStopper", "MaximumIterationStopper", "TrialPlateauStopper",
           "ExperimentPlateauStopper", "TimeoutStopper", "CombinedStopper"]
