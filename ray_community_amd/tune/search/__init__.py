"""Search algorithms (reference: ``python/ray/tune/search``)."""
from __future__ import annotations

import copy
import itertools
import random
from typing import Any, Dict, List, Optional

import numpy as np

from .sample import Domain, Function

UNRESOLVED_SEARCH_SPACE = "unresolved"


def _walk(d, prefix=()):
    if isinstance(d, dict):
        if set(d.keys()) == {"grid_search"}:
            yield prefix, d
            return
        for k, v in d.items():
            yield from _walk(v, prefix + (k,))
    elif isinstance(d, (list, tuple)) and any(isinstance(x, (dict, Domain)) for x in d):
        for i, v in enumerate(d):
            yield from _walk(v, prefix + (i,))
    else:
        yield prefix, d


def _set(d, path, value):
    for k in path[:-1]:
        d = d[k]
    d[path[-1]] = value


def _get(d, path):
    for k in path:
        d = d[k]
    return d


class Searcher:
    FINISHED = "FINISHED"

    def __init__(self, metric: Optional[str] = None, mode: Optional[str] = None):
        self._metric = metric
        self._mode = mode

    @property
    def metric(self):
        return self._metric

    @property
    def mode(self):
        return self._mode

    def set_search_properties(self, metric, mode, config, **spec):
        if self._metric is None:
            self._metric = metric
        if self._mode is None:
            self._mode = mode
        return True

    def suggest(self, trial_id: str) -> Optional[Dict]:
        raise NotImplementedError

    def on_trial_result(self, trial_id: str, result: Dict):
        pass

    def on_trial_complete(self, trial_id: str, result: Optional[Dict] = None, error: bool = False):
        pass

    def save(self, path):
        """Pickle ``get_state()`` to ``path`` (searchers with extra state override get/set_state)."""
        import pickle

        import cloudpickle

        with open(path, "wb") as f:
            cloudpickle.dump(self.get_state(), f)

    def restore(self, path):
        import pickle

        with open(path, "rb") as f:  # a file this framework's save() wrote
            self.set_state(pickle.load(f))

    def get_state(self) -> Dict:
        """The searcher's picklable attributes (modules, locks and the like are left out)."""
        import cloudpickle

        out = {}
        for k, v in self.__dict__.items():
            try:
                cloudpickle.dumps(v)
            except Exception:
                continue
            out[k] = v
        return out

    def set_state(self, state: Dict) -> None:
        self.__dict__.update(state)

    CKPT_FILE_TMPL = "searcher-state-{}.pkl"

    def save_to_dir(self, checkpoint_dir: str, session_str: str = "default") -> None:
        import os

        self.save(os.path.join(checkpoint_dir, self.CKPT_FILE_TMPL.format(session_str)))

    def restore_from_dir(self, checkpoint_dir: str) -> None:
        import glob
        import os

        files = sorted(glob.glob(os.path.join(checkpoint_dir, self.CKPT_FILE_TMPL.format("*"))))
        if not files:
            raise RuntimeError(f"no searcher checkpoint in {checkpoint_dir}")
        self.restore(files[-1])

    def set_max_concurrency(self, max_concurrent: int) -> bool:
        """Searchers that limit concurrency themselves return True (the default lets a
        ConcurrencyLimiter wrap them)."""
        return False

    def add_evaluated_point(self, parameters: Dict, value: float, error: bool = False, pruned: bool = False,
                            intermediate_values=None) -> None:
        """Seed the searcher with a finished evaluation (reference API). Searchers that learn from
        history override this; the base records it and replays it as a completed trial."""
        import uuid

        tid = "evaluated_" + uuid.uuid4().hex[:8]
        self._evaluated = getattr(self, "_evaluated", []) + [(dict(parameters), value)]
        self.on_trial_complete(tid, result={**dict(parameters), **({self._metric: value} if self._metric else {}),
                                            "config": dict(parameters)}, error=error)

    def add_evaluated_trials(self, trials_or_analysis, metric: str) -> None:
        """Seed from finished trials / a ResultGrid: each result's config and ``metric``."""
        items = list(trials_or_analysis)
        for t in items:
            cfg = getattr(t, "config", None) or {}
            res = getattr(t, "metrics", None) or getattr(t, "last_result", None) or {}
            if metric in res:
                self.add_evaluated_point(cfg, res[metric])


def generate_variants(spec: Dict, num_samples: int = 1, rng=None) -> List[Dict]:
    """Grid search cross product x num_samples, then resolve every Domain (sample_from last)."""
    rng = rng or np.random
    grid_axes = [(p, v["grid_search"]) for p, v in _walk(spec) if isinstance(v, dict) and "grid_search" in v]
    combos = list(itertools.product(*[vals for _, vals in grid_axes])) if grid_axes else [()]
    out = []
    for _ in range(num_samples):
        for combo in combos:
            cfg = copy.deepcopy(spec)
            for (p, _), val in zip(grid_axes, combo):
                _set(cfg, p, val)
            funcs = []
            for p, v in _walk(cfg):
                if isinstance(v, Function):
                    funcs.append((p, v))
                elif isinstance(v, Domain):
                    _set(cfg, p, v.sample(random_state=rng))
            for p, v in funcs:
                _set(cfg, p, v.sample(spec=_Spec(cfg), random_state=rng))
            out.append(cfg)
    return out


class _Spec(dict):
    """Lets sample_from lambdas use ``spec.config.x`` like the reference."""

    def __init__(self, cfg):
        super().__init__(config=cfg)
        self.config = _AttrDict(cfg)


class _AttrDict(dict):
    def __getattr__(self, k):
        v = self[k]
        return _AttrDict(v) if isinstance(v, dict) else v


class BasicVariantGenerator(Searcher):
    def __init__(self, points_to_evaluate: Optional[List[Dict]] = None, max_concurrent: int = 0,
                 constant_grid_search: bool = False, random_state=None):
        super().__init__()
        self._points = list(points_to_evaluate or [])
        self._queue: List[Dict] = []
        self._rng = np.random.RandomState(random_state) if random_state is not None else np.random
        self.max_concurrent = max_concurrent
        self._finished = False

    def set_space(self, param_space: Dict, num_samples: int):
        self._queue = list(self._points) + generate_variants(param_space, num_samples, self._rng)
        self._total = len(self._queue)

    def total(self):
        return len(self._queue)

    @property
    def total_samples(self) -> int:
        """Configurations this generator was given (the initial queue length)."""
        return getattr(self, "_total", len(self._queue))

    def add_configurations(self, experiments) -> None:
        """Queue the variants of more experiments: ``Experiment`` objects, ``{name: spec}`` dicts
        or specs with ``config`` / ``num_samples``."""
        if isinstance(experiments, dict) and "config" not in experiments:
            experiments = list(experiments.values())
        for e in (experiments if isinstance(experiments, (list, tuple)) else [experiments]):
            cfg = getattr(e, "config", None) if not isinstance(e, dict) else e.get("config")
            n = getattr(e, "num_samples", None) if not isinstance(e, dict) else e.get("num_samples", 1)
            new = generate_variants(cfg or {}, int(n or 1), self._rng)
            self._queue.extend(new)
            self._total = self.total_samples + len(new)

    def next_trial(self) -> Optional[Dict]:
        """The next configuration, or None when the generator is exhausted."""
        return self._queue.pop(0) if self._queue else None

    def has_checkpoint(self, dirpath: str) -> bool:
        return False

    def suggest(self, trial_id):
        if not self._queue:
            return Searcher.FINISHED
        return self._queue.pop(0)


class ConcurrencyLimiter(Searcher):
    """At most ``max_concurrent`` live trials. ``batch=True``: suggestions come in batches of
    ``max_concurrent``; the next batch starts once every trial of the current one completed, and
    the wrapped searcher sees the batch's results together (reference
    tune/search/concurrency_limiter.py)."""

    def __init__(self, searcher: Searcher, max_concurrent: int, batch: bool = False):
        super().__init__(searcher.metric, searcher.mode)
        if max_concurrent < 1:
            raise ValueError("max_concurrent must be >= 1")
        self.searcher = searcher
        self.max_concurrent = max_concurrent
        self.batch = batch
        self.live = set()
        self._paused = set()
        self._batch_full = False
        self._cached: List[tuple] = []

    def set_search_properties(self, metric, mode, config, **spec):
        return self.searcher.set_search_properties(metric, mode, config, **spec)

    def suggest(self, trial_id):
        if len(self.live) >= self.max_concurrent or (self.batch and self._batch_full):
            return None
        s = self.searcher.suggest(trial_id)
        if s is not None and s != Searcher.FINISHED:
            self.live.add(trial_id)
            if self.batch and len(self.live) >= self.max_concurrent:
                self._batch_full = True
        return s

    def on_trial_result(self, trial_id, result):
        self.searcher.on_trial_result(trial_id, result)

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.live.discard(trial_id)
        self._paused.discard(trial_id)
        if not self.batch:
            self.searcher.on_trial_complete(trial_id, result, error)
            return
        self._cached.append((trial_id, result, error))
        if not self.live:  # the whole batch is done: report it and open the next one
            for tid, res, err in self._cached:
                self.searcher.on_trial_complete(tid, res, err)
            self._cached = []
            self._batch_full = False

    def on_pause(self, trial_id) -> None:
        """A paused trial frees its slot (schedulers pause trials at milestones)."""
        if trial_id in self.live:
            self.live.discard(trial_id)
            self._paused.add(trial_id)

    def on_unpause(self, trial_id) -> None:
        if trial_id in self._paused:
            self._paused.discard(trial_id)
            self.live.add(trial_id)


class RandomSearch(Searcher):
    """Independent random sampling from a space of Domains (the unit for model-based searchers)."""

    def __init__(self, space: Optional[Dict] = None, metric=None, mode=None, seed=None):
        super().__init__(metric, mode)
        self.space = space
        self._rng = np.random.RandomState(seed)

    def set_search_properties(self, metric, mode, config, **spec):
        super().set_search_properties(metric, mode, config)
        if self.space is None:
            self.space = config
        return True

    def suggest(self, trial_id):
        return generate_variants(self.space, 1, self._rng)[0]


TRIAL_INDEX = "__trial_index__"


class Repeater(Searcher):
    """Evaluates every configuration of the wrapped searcher ``repeat`` times (reference
    ``tune/search/repeater.py``): the copies carry ``config[TRIAL_INDEX]`` = 0..repeat-1 when
    ``set_index``, and once all copies of a configuration completed the wrapped searcher is told
    ONE completion with the mean of their ``metric`` (so model-based searchers see averaged,
    less noisy scores)."""

    def __init__(self, searcher: Searcher, repeat: int = 1, set_index: bool = True):
        super().__init__(searcher.metric, searcher.mode)
        self.searcher = searcher
        self.repeat = max(1, int(repeat))
        self.set_index = set_index
        self._current = None
        self._left = 0
        self._group = -1
        self._group_of: Dict[str, int] = {}
        self._groups: Dict[int, Dict] = {}  # group -> {"first": trial id, "scores": [...], "done": n}

    def set_search_properties(self, metric, mode, config, **spec):
        super().set_search_properties(metric, mode, config)
        return self.searcher.set_search_properties(metric, mode, config, **spec)

    def suggest(self, trial_id):
        if self._left == 0:
            cfg = self.searcher.suggest(trial_id)
            if cfg is None or cfg == Searcher.FINISHED:
                return cfg
            self._current = cfg
            self._left = self.repeat
            self._group += 1
            self._groups[self._group] = {"first": trial_id, "scores": [], "done": 0}
        idx = self.repeat - self._left
        self._left -= 1
        self._group_of[trial_id] = self._group
        cfg = copy.deepcopy(self._current)
        if self.set_index and isinstance(cfg, dict):
            cfg[TRIAL_INDEX] = idx
        return cfg

    def on_trial_complete(self, trial_id, result=None, error=False):
        g = self._group_of.pop(trial_id, None)
        if g is None:
            return
        st = self._groups[g]
        st["done"] += 1
        metric = self.searcher.metric or self.metric
        if result and metric in result and not error:
            st["scores"].append(float(result[metric]))
        if st["done"] == self.repeat:
            self._groups.pop(g)
            mean = float(np.nanmean(st["scores"])) if st["scores"] else float("nan")
            self.searcher.on_trial_complete(st["first"], {metric: mean} if metric else None,
                                            error=not st["scores"])


UNDEFINED_SEARCH_SPACE = "Trying to sample a configuration from {cls}, but no search space has been defined."
UNDEFINED_METRIC_MODE = "Trying to sample a configuration from {cls}, but the `metric` ({metric}) or `mode` ({mode})" \
                        " parameters have not been set."


class SearchAlgorithm:
    """Trial-producing interface (reference ``tune/search/search_algorithm.py``); every Searcher
    is driven through it by ``SearchGenerator``."""

    def set_search_properties(self, metric, mode, config, **spec) -> bool:
        return True

    def next_trial(self):
        raise NotImplementedError

    def on_trial_result(self, trial_id, result):
        pass

    def on_trial_complete(self, trial_id, result=None, error=False):
        pass

    def is_finished(self) -> bool:
        return False


class SearchGenerator(SearchAlgorithm):
    """Adapts a ``Searcher`` (suggest-style) to the SearchAlgorithm interface."""

    def __init__(self, searcher: Searcher):
        self.searcher = searcher
        self._finished = False
        self._n = 0

    def set_search_properties(self, metric, mode, config, **spec):
        ok = self.searcher.set_search_properties(metric, mode, config, **spec)
        if hasattr(self.searcher, "set_space") and config:
            self.searcher.set_space(config, int(spec.get("num_samples", 1)))
        return ok

    def next_trial(self):
        self._n += 1
        cfg = self.searcher.suggest(f"trial_{self._n:05d}")
        if cfg == Searcher.FINISHED:
            self._finished = True
            return None
        return cfg

    def on_trial_result(self, trial_id, result):
        self.searcher.on_trial_result(trial_id, result)

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.searcher.on_trial_complete(trial_id, result, error)

    def is_finished(self):
        return self._finished


def __getattr__(name):
    if name == "grid_search":
        from .sample import grid_search

        return grid_search
    if name in ("TPESearch", "OptunaSearch", "HyperOptSearch"):
        from . import tpe

        return getattr(tpe, name)
    if name == "TuneBOHB":
        from .bohb import TuneBOHB

        return TuneBOHB
    raise AttributeError(name)


__all__ = ["Searcher", "BasicVariantGenerator", "ConcurrencyLimiter", "RandomSearch", "Repeater",
           "generate_variants", "TPESearch", "OptunaSearch", "HyperOptSearch", "TuneBOHB", "SearchAlgorithm", "SearchGenerator",
           "grid_search", "UNDEFINED_SEARCH_SPACE", "UNDEFINED_METRIC_MODE"]
