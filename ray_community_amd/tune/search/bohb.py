"""BOHB searcher (Falkner et al. 2018; reference ``python/ray/tune/search/bohb/bohb_search.py``,
which wraps hpbandster -- not installable here, so this is a native implementation on the TPE
density models of ``tpe.py``).

Paired with ``HyperBandForBOHB``: every intermediate result is an observation at a BUDGET
(``time_attr``, e.g. training_iteration). A suggestion fits the good / bad Parzen models on the
LARGEST budget that has at least ``min_points_in_model`` observations (falling back to random
sampling until one does), and a ``random_fraction`` of suggestions stays random, as in BOHB.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import numpy as np

from . import generate_variants
from .tpe import TPESearch


class TuneBOHB(TPESearch):
    def __init__(self, space: Optional[Dict] = None, metric: Optional[str] = None, mode: Optional[str] = None,
                 points_to_evaluate: Optional[List[Dict]] = None, seed: Optional[int] = None,
                 time_attr: str = "training_iteration", min_points_in_model: Optional[int] = None,
                 top_n_percent: int = 15, random_fraction: float = 1 / 3, num_samples: int = 64, **kw):
        super().__init__(space, metric, mode, points_to_evaluate, n_startup_trials=0,
                         gamma=top_n_percent / 100.0, n_ei_candidates=num_samples, seed=seed)
        self._time_attr = time_attr
        self._min_points = min_points_in_model
        self._random_fraction = random_fraction
        self._by_budget: Dict[float, Dict[str, tuple]] = {}  # budget -> trial -> (flat params, score)
        self.model_budgets: List[Optional[float]] = []      # budget each suggestion was modelled on

    def _flat(self, cfg):
        flat = {}
        for path, _ in self._params():
            try:
                v = cfg
                for k in path:
                    v = v[k]
                flat[path] = v
            except (KeyError, IndexError, TypeError):
                pass
        return flat

    def on_trial_result(self, trial_id, result):
        cfg = self._live.get(trial_id)
        if cfg is None or self._metric not in result or self._time_attr not in result:
            return
        b = float(result[self._time_attr])
        self._by_budget.setdefault(b, {})[trial_id] = (self._flat(cfg), float(result[self._metric]))

    def on_trial_complete(self, trial_id, result=None, error=False):
        if result and not error:
            self.on_trial_result(trial_id, result)
        self._live.pop(trial_id, None)

    def suggest(self, trial_id):
        if self._space is None:
            return None
        if self._points:
            cfg = self._points.pop(0)
            self._live[trial_id] = cfg
            return copy.deepcopy(cfg)
        need = self._min_points or (len(self._params()) + 1)
        budgets = sorted((b for b, obs in self._by_budget.items() if len(obs) >= need), reverse=True)
        if not budgets or self._rng.rand() < self._random_fraction:
            self.model_budgets.append(None)
            cfg = generate_variants(self._space, 1, self._rng)[0]
            self._live[trial_id] = cfg
            return copy.deepcopy(cfg)
        b = budgets[0]
        self.model_budgets.append(b)
        self._obs = list(self._by_budget[b].values())
        self._n_startup = 0
        cfg = super().suggest(trial_id)
        return cfg


BOHB = TuneBOHB  # the short name of the reference package
