"""Gaussian-process Bayesian optimisation searcher (reference:
``python/ray/tune/search/bayesopt/bayesopt_search.py``, which wraps the ``bayesian-optimization``
package -- not installed here; this is a native implementation on scikit-learn's GP regressor).

The search space is continuous: ``{"x": (low, high)}`` bounds or ``tune.uniform`` /
``tune.loguniform`` domains (log domains are modelled in log space), nested dicts flattened to
``"a/b"`` keys; constants pass through unchanged. The first ``random_search_steps`` trials are
uniform random and the searcher waits for them to finish; after that every suggestion maximises
the acquisition function over a GP (Matern 5/2 kernel, inputs scaled to the unit cube, targets
normalised) fitted on every finished trial: ``ucb`` (mean + kappa * std, the default), ``ei``
(expected improvement over the best value + xi) or ``poi`` (probability of improvement).
The acquisition is maximised by scoring random candidates and refining the best few with
L-BFGS-B. Suggestions already evaluated (to ``repeat_float_precision`` digits) are skipped; once
one configuration has been suggested more than ``patience`` times the search ends
(``Searcher.FINISHED``), as in the reference.
"""
from __future__ import annotations

import copy
import math
import warnings
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import Searcher
from .sample import Domain, Float


def _flatten(d: Dict, prefix: str = "") -> Dict:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict) and v and not isinstance(v, Domain):
            out.update(_flatten(v, key + "/"))
        else:
            out[key] = v
    return out


def _unflatten(flat: Dict) -> Dict:
    out: Dict = {}
    for k, v in flat.items():
        node = out
        parts = k.split("/")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return out


class BayesOptSearch(Searcher):
    def __init__(self, space: Optional[Dict] = None, metric: Optional[str] = None, mode: Optional[str] = None,
                 points_to_evaluate: Optional[List[Dict]] = None, utility_kwargs: Optional[Dict] = None,
                 random_state: int = 42, random_search_steps: int = 10, verbose: int = 0, patience: int = 5,
                 skip_duplicate: bool = True, analysis=None, n_candidates: int = 4000):
        super().__init__(metric, mode)
        if mode not in (None, "min", "max"):
            raise ValueError("`mode` must be 'min' or 'max'")
        self._utility = {"kind": "ucb", "kappa": 2.576, "xi": 0.0, **(utility_kwargs or {})}
        if self._utility["kind"] not in ("ucb", "ei", "poi"):
            raise ValueError(f"utility kind must be ucb, ei or poi; got {self._utility['kind']!r}")
        self._points = [_flatten(p) for p in (points_to_evaluate or [])]
        self.random_search_trials = int(random_search_steps)
        self._patience = patience
        self._skip_duplicate = skip_duplicate
        self.repeat_float_precision = 5
        self._rng = np.random.RandomState(random_state)
        self._seed = random_state
        self._n_cand = int(n_candidates)
        self._verbose = verbose
        self._names: List[str] = []
        self._bounds = np.zeros((0, 2))
        self._log = np.zeros(0, dtype=bool)
        self._const: Dict = {}
        self._live: Dict[str, Dict] = {}
        self._X: List[np.ndarray] = []  # unit-cube inputs of finished trials
        self._y: List[float] = []       # their targets, sign-adjusted so larger is better
        self._counter: Dict[tuple, int] = defaultdict(int)
        self._random_issued = 0
        self._space_set = False
        if space:
            self._set_space(space)
        if analysis is not None:
            self.register_analysis(analysis)

    # ------------------------------------------------------------------ space
    def _set_space(self, space: Dict):
        names, bounds, log, const = [], [], [], {}
        for k, v in _flatten(space).items():
            if isinstance(v, (tuple, list)) and len(v) == 2 and all(isinstance(x, (int, float)) for x in v):
                lo, hi, lg = float(v[0]), float(v[1]), False
            elif isinstance(v, Float):
                lo, hi, lg = float(v.lower), float(v.upper), bool(v.log)
                if getattr(v, "normal", False):
                    raise ValueError(f"BayesOpt does not support normal-distributed parameters ({k})")
            elif isinstance(v, Domain):
                raise ValueError(f"BayesOpt only supports continuous float parameters; {k!r} is "
                                 f"{type(v).__name__}")
            else:
                const[k] = v
                continue
            if not hi > lo:
                raise ValueError(f"empty range for {k!r}: ({lo}, {hi})")
            if lg:
                lo, hi = math.log(lo), math.log(hi)
            names.append(k)
            bounds.append((lo, hi))
            log.append(lg)
        if not names:
            raise ValueError("BayesOptSearch needs at least one continuous parameter")
        self._names, self._bounds, self._log, self._const = names, np.asarray(bounds), np.asarray(log), const
        self._space_set = True

    def set_search_properties(self, metric, mode, config, **spec):
        if self._space_set:
            return False
        super().set_search_properties(metric, mode, config)
        if config:
            self._set_space(config)
        return True

    def _to_unit(self, flat: Dict) -> np.ndarray:
        x = np.array([float(flat[n]) for n in self._names])
        x = np.where(self._log, np.log(np.maximum(x, 1e-300)), x)
        lo, hi = self._bounds[:, 0], self._bounds[:, 1]
        return np.clip((x - lo) / (hi - lo), 0.0, 1.0)

    def _from_unit(self, u: np.ndarray) -> Dict:
        lo, hi = self._bounds[:, 0], self._bounds[:, 1]
        x = lo + np.clip(u, 0.0, 1.0) * (hi - lo)
        x = np.where(self._log, np.exp(x), x)
        flat = {n: float(v) for n, v in zip(self._names, x)}
        flat.update(self._const)
        return flat

    # ------------------------------------------------------------------ GP + acquisition
    def _fit(self):
        from sklearn.gaussian_process import GaussianProcessRegressor
        from sklearn.gaussian_process.kernels import ConstantKernel, Matern

        gp = GaussianProcessRegressor(kernel=ConstantKernel(1.0, (1e-3, 1e3)) * Matern(
            length_scale=np.full(len(self._names), 0.5), length_scale_bounds=(1e-3, 1e2), nu=2.5),
            alpha=1e-6, normalize_y=True, n_restarts_optimizer=3, random_state=self._seed)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            gp.fit(np.stack(self._X), np.asarray(self._y))
        return gp

    def _acq(self, gp, U: np.ndarray, best: float) -> np.ndarray:
        from scipy.stats import norm

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            mu, sd = gp.predict(U, return_std=True)
        kind = self._utility["kind"]
        if kind == "ucb":
            return mu + self._utility["kappa"] * sd
        sd = np.maximum(sd, 1e-9)
        z = (mu - best - self._utility["xi"]) / sd
        if kind == "ei":
            return (mu - best - self._utility["xi"]) * norm.cdf(z) + sd * norm.pdf(z)
        return norm.cdf(z)

    def _maximize(self) -> np.ndarray:
        from scipy.optimize import minimize

        gp = self._fit()
        best = max(self._y)
        d = len(self._names)
        U = self._rng.uniform(size=(self._n_cand, d))
        a = self._acq(gp, U, best)
        top = U[np.argsort(-a)[:3]]
        x_best, a_best = U[int(np.argmax(a))], float(a.max())
        for x0 in top:
            r = minimize(lambda x: -float(self._acq(gp, x[None], best)[0]), x0, method="L-BFGS-B",
                         bounds=[(0.0, 1.0)] * d)
            if r.success and -float(r.fun) > a_best:
                x_best, a_best = np.clip(r.x, 0.0, 1.0), -float(r.fun)
        return x_best

    # ------------------------------------------------------------------ Searcher API
    def _key(self, flat: Dict) -> tuple:
        return tuple((n, round(float(flat[n]), self.repeat_float_precision)) for n in self._names)

    def suggest(self, trial_id: str) -> Optional[Dict]:
        if not self._space_set:
            raise RuntimeError("BayesOptSearch has no search space: pass `space` or a param_space to the Tuner")
        if not self._metric or not self._mode:
            raise RuntimeError("BayesOptSearch needs `metric` and `mode` (here or in the TuneConfig)")
        # warm-up: the first random_search_steps suggestions (points_to_evaluate included) are not
        # modelled, and the GP waits until that many trials have finished
        random_phase = len(self._y) < self.random_search_trials
        if random_phase and self._random_issued >= self.random_search_trials:
            return None
        if self._points:
            flat = dict(self._points.pop(0))
            flat.update({k: v for k, v in self._const.items() if k not in flat})
        elif random_phase:
            flat = self._from_unit(self._rng.uniform(size=len(self._names)))
        else:
            flat = self._from_unit(self._maximize())
        key = self._key(flat)
        seen = key in self._counter
        self._counter[key] += 1
        if self._patience is not None and max(self._counter.values()) > self._patience:
            return Searcher.FINISHED
        if seen and self._skip_duplicate:
            return None
        if random_phase:
            self._random_issued += 1
        self._live[trial_id] = flat
        return copy.deepcopy(_unflatten(flat))

    def _observe(self, flat: Dict, value: float):
        if value is None or not np.isfinite(value):
            return
        self._X.append(self._to_unit(flat))
        self._y.append(float(value) if self._mode == "max" else -float(value))

    def on_trial_complete(self, trial_id: str, result: Optional[Dict] = None, error: bool = False):
        flat = self._live.pop(trial_id, None)
        if flat is None or error or not result or self._metric not in result:
            return
        self._observe(flat, float(result[self._metric]))

    def register_analysis(self, analysis):
        """Add the trials of an earlier experiment (an ExperimentAnalysis) to the GP's data."""
        if not self._space_set:
            raise RuntimeError("register_analysis needs the search space first")
        for t in analysis.trials:
            res = t.last_result or {}
            if self._metric in res:
                flat = _flatten(t.config)
                if all(n in flat for n in self._names):
                    self._observe(flat, float(res[self._metric]))

    def get_state(self) -> Dict:
        st = super().get_state()
        st["_counter"] = dict(self._counter)
        return st

    def set_state(self, state: Dict) -> None:
        state = dict(state)
        state["_counter"] = defaultdict(int, state.get("_counter") or {})
        super().set_state(state)


__all__ = ["BayesOptSearch"]
