"""Tree-structured Parzen Estimator searcher (native; the reference delegates to Optuna /
HyperOpt, which are not installable here — reference: ``python/ray/tune/search/optuna``,
``hyperopt``; algorithm: Bergstra et al. 2011).

Each numeric parameter is modelled in its own transformed space (log for log domains) by two
Parzen mixtures — over the best ``gamma`` fraction of finished trials (l) and the rest (g) — and
categoricals by smoothed frequencies. After ``n_startup_trials`` random trials, each suggestion is
the candidate (sampled from l) that maximises l(x) / g(x).
"""
from __future__ import annotations

import copy
import math
from typing import Dict, List, Optional

import numpy as np

from . import Searcher, _set, _walk, generate_variants
from .sample import Categorical, Domain, Float, Integer


class TPESearch(Searcher):
    def __init__(self, space: Optional[Dict] = None, metric: Optional[str] = None, mode: Optional[str] = None,
                 points_to_evaluate: Optional[List[Dict]] = None, n_startup_trials: int = 10, gamma: float = 0.25,
                 n_ei_candidates: int = 24, seed: Optional[int] = None):
        super().__init__(metric, mode)
        self._space = space
        self._points = list(points_to_evaluate or [])
        self._n_startup = n_startup_trials
        self._gamma = gamma
        self._n_cand = n_ei_candidates
        self._rng = np.random.RandomState(seed)
        self._live: Dict[str, Dict] = {}
        self._obs: List = []  # (flat params dict, score)

    def set_search_properties(self, metric, mode, config, **spec):
        super().set_search_properties(metric, mode, config)
        if self._space is None:
            self._space = config
        return True

    def _params(self):
        return [(p, d) for p, d in _walk(self._space) if isinstance(d, Domain)]

    # ----------------------------------------------------------------- per-parameter models
    @staticmethod
    def _to_unit(d, v):
        if isinstance(d, (Float, Integer)) and d.log:
            return math.log(v)
        return float(v)

    @staticmethod
    def _bounds(d):
        lo, hi = float(d.lower), float(d.upper)
        if d.log:
            return math.log(lo), math.log(hi)
        return lo, hi

    def _parzen(self, xs, lo, hi):
        xs = np.asarray(xs, dtype=np.float64)
        if len(xs) == 0:
            return np.array([(lo + hi) / 2]), np.array([hi - lo])
        bw = max((hi - lo) / max(1.0, len(xs)) ** 0.8, 1e-3 * (hi - lo))
        mus = np.concatenate([xs, [(lo + hi) / 2]])
        sig = np.concatenate([np.full(len(xs), bw), [hi - lo]])
        return mus, sig

    @staticmethod
    def _logpdf(x, mus, sig):
        z = (x[:, None] - mus[None, :]) / sig[None, :]
        lp = -0.5 * z * z - np.log(sig[None, :] * math.sqrt(2 * math.pi))
        m = lp.max(1, keepdims=True)
        return (m + np.log(np.exp(lp - m).mean(1, keepdims=True)))[:, 0]

    def _suggest_numeric(self, d, good, bad):
        lo, hi = self._bounds(d)
        mg, sg = self._parzen([self._to_unit(d, v) for v in good], lo, hi)
        mb, sb = self._parzen([self._to_unit(d, v) for v in bad], lo, hi)
        idx = self._rng.randint(len(mg), size=self._n_cand)
        cand = np.clip(self._rng.normal(mg[idx], sg[idx]), lo, hi)
        score = self._logpdf(cand, mg, sg) - self._logpdf(cand, mb, sb)
        return cand, score

    def _finalize(self, d, u):
        v = math.exp(u) if d.log else u
        if isinstance(d, Integer):
            v = int(round(v))
            hi = d.upper if d.q else d.upper - 1
            return int(min(max(v, d.lower), hi))
        if d.q:
            v = round(v / d.q) * d.q
        return float(min(max(v, d.lower), d.upper))

    def suggest(self, trial_id):
        if self._space is None:
            return None
        if self._points:
            cfg = self._points.pop(0)
            self._live[trial_id] = cfg
            return copy.deepcopy(cfg)
        cfg = generate_variants(self._space, 1, self._rng)[0]
        done = [o for o in self._obs if o[1] is not None and np.isfinite(o[1])]
        if len(done) >= self._n_startup:
            sign = -1.0 if self._mode == "max" else 1.0
            ranked = sorted(done, key=lambda o: sign * o[1])
            n_good = max(1, int(math.ceil(self._gamma * len(ranked))))
            good, bad = ranked[:n_good], ranked[n_good:]
            for path, d in self._params():
                key = path
                gv = [o[0][key] for o in good if key in o[0]]
                bv = [o[0][key] for o in bad if key in o[0]]
                if isinstance(d, Categorical):
                    cats = d.categories
                    w_g = np.array([1.0 + sum(1 for v in gv if v == c) for c in cats])
                    w_b = np.array([1.0 + sum(1 for v in bv if v == c) for c in cats])
                    ratio = (w_g / w_g.sum()) / (w_b / w_b.sum())
                    _set(cfg, path, cats[int(np.argmax(ratio))])
                elif isinstance(d, (Float, Integer)) and not getattr(d, "normal", False):
                    cand, score = self._suggest_numeric(d, gv, bv)
                    _set(cfg, path, self._finalize(d, float(cand[int(np.argmax(score))])))
        self._live[trial_id] = cfg
        return copy.deepcopy(cfg)

    def on_trial_complete(self, trial_id, result=None, error=False):
        cfg = self._live.pop(trial_id, None)
        if cfg is None or error or not result or self._metric not in result:
            return
        flat = {}
        for path, _ in self._params():
            try:
                v = cfg
                for k in path:
                    v = v[k]
                flat[path] = v
            except (KeyError, IndexError, TypeError):
                pass
        self._obs.append((flat, float(result[self._metric])))


class OptunaSearch(TPESearch):
    """Name-compatible alias: Optuna's default sampler is TPE; this is the native implementation."""


class HyperOptSearch(TPESearch):
    """Name-compatible alias: HyperOpt's main algorithm is TPE; this is the native implementation."""
