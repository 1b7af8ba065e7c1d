"""Population Based Bandits (reference: ``python/ray/tune/schedulers/pb2.py``; Parker-Holder et
al. 2020). PBT's exploit step, with the explore step replaced by GP-UCB: a Gaussian process
(scikit-learn, Matern kernel) models the per-interval improvement of the metric as a function of
(time, hyperparameters) over the whole population, and the new configuration for a cloned trial
is the UCB-maximising point among random candidates inside ``hyperparam_bounds``."""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import numpy as np

from . import PopulationBasedTraining


class PB2(PopulationBasedTraining):
    def __init__(self, time_attr="training_iteration", metric=None, mode=None, perturbation_interval=60.0,
                 hyperparam_bounds: Optional[Dict[str, List[float]]] = None, quantile_fraction=0.25, log_config=True,
                 require_attrs=True, synch=False, custom_explore_fn=None, n_candidates: int = 256, kappa: float = 2.0,
                 seed=None):
        if not hyperparam_bounds:
            raise ValueError("`hyperparam_bounds` must be specified for PB2")
        for k, (lo, hi) in hyperparam_bounds.items():
            if not lo < hi:
                raise ValueError(f"invalid bounds for {k}: {lo} >= {hi}")
        self.bounds = {k: (float(v[0]), float(v[1])) for k, v in hyperparam_bounds.items()}
        mutations = {k: (lambda lo=lo, hi=hi: float(np.random.uniform(lo, hi))) for k, (lo, hi) in self.bounds.items()}
        super().__init__(time_attr=time_attr, metric=metric, mode=mode, perturbation_interval=perturbation_interval,
                         hyperparam_mutations=mutations, quantile_fraction=quantile_fraction,
                         resample_probability=0.0, custom_explore_fn=custom_explore_fn, seed=seed)
        self.n_candidates = n_candidates
        self.kappa = kappa
        self._np_rng = np.random.RandomState(seed)
        self._last: Dict[str, tuple] = {}  # trial -> (t, score)
        self._X: List[List[float]] = []
        self._y: List[float] = []
        self._configs: Dict[str, Dict] = {}

    def _vec(self, config) -> List[float]:
        return [(float(config.get(k, (lo + hi) / 2)) - lo) / (hi - lo) for k, (lo, hi) in self.bounds.items()]

    def on_trial_result(self, controller, trial, result):
        t = result.get(self.time_attr)
        s = self._score(result)
        if t is not None and s is not None:
            prev = self._last.get(trial.trial_id)
            if prev is not None and t > prev[0]:
                self._X.append([float(t)] + self._vec(trial.config))
                self._y.append((s - prev[1]) / (t - prev[0]))
            self._last[trial.trial_id] = (t, s)
        return super().on_trial_result(controller, trial, result)

    def _explore(self, config):
        new = copy.deepcopy(config)
        keys = list(self.bounds)
        if len(self._y) < 3:
            for k, (lo, hi) in self.bounds.items():
                new[k] = float(self._np_rng.uniform(lo, hi))
            return self.custom_explore_fn(new) if self.custom_explore_fn else new
        from sklearn.gaussian_process import GaussianProcessRegressor
        from sklearn.gaussian_process.kernels import Matern, WhiteKernel

        X = np.asarray(self._X[-500:], dtype=np.float64)
        y = np.asarray(self._y[-500:], dtype=np.float64)
        tmax = max(X[:, 0].max(), 1.0)
        X[:, 0] /= tmax
        ys = (y - y.mean()) / (y.std() + 1e-9)
        gp = GaussianProcessRegressor(kernel=Matern(nu=2.5) + WhiteKernel(1e-3), normalize_y=False,
                                      random_state=int(self._np_rng.randint(1 << 30)))
        gp.fit(X, ys)
        cand = self._np_rng.uniform(0, 1, size=(self.n_candidates, len(keys)))
        tcol = np.full((self.n_candidates, 1), X[:, 0].max())
        mu, sd = gp.predict(np.hstack([tcol, cand]), return_std=True)
        best = cand[int(np.argmax(mu + self.kappa * sd))]
        for k, u in zip(keys, best):
            lo, hi = self.bounds[k]
            new[k] = float(lo + u * (hi - lo))
        return self.custom_explore_fn(new) if self.custom_explore_fn else new


def import_pb2_dependencies():
    """(GPy, sklearn) in the reference; the GP here is sklearn's, so GPy is None."""
    try:
        import sklearn
    except ImportError:
        sklearn = None
    return None, sklearn
