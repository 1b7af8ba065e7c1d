"""Named trainables / envs, ``Experiment`` specs and progress reporters (reference:
``python/ray/tune/registry.py``, ``tune/experiment/experiment.py``, ``tune/progress_reporter.py``,
``tune/execution/placement_groups.py``, ``tune/search/__init__.py::create_searcher``,
``tune/schedulers/__init__.py::create_scheduler``).

``register_trainable(name, fn_or_class)`` makes ``Tuner("name")`` / ``tune.run("name")`` work;
``register_env`` is RLlib's env registry (``rllib/env/envs.py``). Reporters print a trial table
(status, iteration, last metrics) every ``max_report_frequency`` seconds and on completion through
the Tuner's callback hooks.
"""
from __future__ import annotations

import sys
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Union

_TRAINABLES: Dict[str, Any] = {}


def register_trainable(name: str, trainable, warn: bool = True):
    if not callable(trainable):
        raise TypeError(f"{trainable!r} is not a trainable (function or Trainable class)")
    _TRAINABLES[name] = trainable


def register_env(name: str, env_creator: Callable):
    from ..rllib.env.envs import register_env as _reg

    _reg(name, env_creator)


def get_trainable_cls(name: str):
    if name not in _TRAINABLES:
        # RLlib algorithms are trainables by name ("PPO", "DQN", ...)
        try:
            from ..rllib.algorithms import get_algorithm_class

            return get_algorithm_class(name)
        except Exception:  # noqa
            raise ValueError(f"Unknown trainable {name!r}: register it with tune.register_trainable")
    return _TRAINABLES[name]


def resolve_trainable(t):
    return get_trainable_cls(t) if isinstance(t, str) else t


class PlacementGroupFactory:
    """Per-trial resource request as placement-group bundles (the first bundle is the trial's own
    actor). Accepted wherever ``tune.with_resources`` takes a dict."""

    def __init__(self, bundles: List[Dict[str, float]], strategy: str = "PACK", *args, **kwargs):
        if not bundles:
            raise ValueError("PlacementGroupFactory needs at least one bundle")
        self.bundles = [{k: float(v) for k, v in b.items()} for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle_is_empty(self):
        return not any(self.bundles[0].values())

    @property
    def required_resources(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0.0) + v
        return out

    def __eq__(self, other):
        return isinstance(other, PlacementGroupFactory) and (self.bundles, self.strategy) == (other.bundles,
                                                                                                other.strategy)

    def __repr__(self):
        return f"PlacementGroupFactory({self.bundles}, strategy={self.strategy!r})"


@dataclass
class Experiment:
    name: str
    run: Any
    stop: Optional[Dict] = None
    config: Dict = field(default_factory=dict)
    resources_per_trial: Optional[Dict] = None
    num_samples: int = 1
    storage_path: Optional[str] = None
    checkpoint_config: Any = None
    max_failures: int = 0

    @classmethod
    def from_json(cls, name: str, spec: Dict) -> "Experiment":
        spec = dict(spec)
        return cls(name=name, run=spec.pop("run"), **spec)


_RUN_EXPERIMENTS_PASSTHROUGH = ("resume", "resume_config", "reuse_actors", "callbacks", "progress_reporter",
                                "trial_name_creator", "trial_dirname_creator", "max_concurrent_trials")


def run_experiments(experiments: Union[Experiment, List[Experiment], Dict[str, Dict]], scheduler=None,
                    verbose: int = 2, raise_on_failed_trial: bool = True, **kw) -> List:
    """Run one or more experiments one after another; returns every trial's result."""
    from . import run as _run

    if isinstance(experiments, dict):
        experiments = [Experiment.from_json(n, s) for n, s in experiments.items()]
    elif isinstance(experiments, Experiment):
        experiments = [experiments]
    trials = []
    for e in experiments:
        ana = _run(resolve_trainable(e.run), name=e.name, stop=e.stop, config=e.config,
                   resources_per_trial=e.resources_per_trial, num_samples=e.num_samples, storage_path=e.storage_path,
                   scheduler=scheduler, checkpoint_config=e.checkpoint_config, max_failures=e.max_failures,
                   raise_on_failed_trial=raise_on_failed_trial, verbose=verbose,
                   **{k: v for k, v in kw.items() if k in _RUN_EXPERIMENTS_PASSTHROUGH})
        trials.extend(ana.trials)
    return trials


def create_searcher(search_alg: str, **kwargs):
    from . import search as S

    table = {"variant_generator": S.BasicVariantGenerator, "random": S.BasicVariantGenerator}
    try:
        from .search import tpe

        for k in ("tpe", "hyperopt", "optuna"):
            table[k] = tpe.TPESearch
    except Exception:  # noqa
        pass
    try:
        from .search.bayesopt import BayesOptSearch

        table["bayesopt"] = BayesOptSearch
    except Exception:  # noqa
        pass
    if search_alg not in table:
        raise ValueError(f"Search algorithm must be one of {sorted(table)}, got {search_alg!r}")
    return table[search_alg](**kwargs)


def create_scheduler(scheduler: str, **kwargs):
    from . import schedulers as S

    table = {"fifo": S.FIFOScheduler, "async_hyperband": S.AsyncHyperBandScheduler, "asynchyperband":
             S.AsyncHyperBandScheduler, "asha": S.ASHAScheduler, "hyperband": S.HyperBandScheduler,
             "median_stopping_rule": S.MedianStoppingRule, "pbt": S.PopulationBasedTraining}
    try:
        from .schedulers.pb2 import PB2

        table["pb2"] = PB2
    except Exception:  # noqa
        pass
    if scheduler not in table:
        raise ValueError(f"Scheduler must be one of {sorted(table)}, got {scheduler!r}")
    return table[scheduler](**kwargs)


@dataclass
class ResumeConfig:
    """What ``Tuner.restore`` does with unfinished / errored trials
    (reference: python/ray/tune/execution/experiment_state.py ResumeConfig)."""

    class ResumeType:
        RESUME = "resume"
        RESTART = "restart"
        SKIP = "skip"

    finished: str = "restore"
    unfinished: str = "resume"
    errored: str = "skip"

    def _restore_kwargs(self) -> Dict:
        """``Tuner.restore`` keyword arguments for this config."""
        return {"resume_unfinished": str(self.unfinished) != "skip",
                "resume_errored": str(self.errored) == "resume",
                "restart_errored": str(self.errored) == "restart"}

    @classmethod
    def _from_legacy(cls, resume) -> Optional["ResumeConfig"]:
        """``tune.run(resume=...)``: True / "AUTO", with an optional "+ERRORED", "+RESTART_ERRORED",
        "+ERRORED_ONLY" or "+RESTART_ERRORED_ONLY" suffix."""
        if resume is False or resume is None:
            return None
        if resume is True:
            return cls()
        head, *suffixes = str(resume).split("+")
        if head != "AUTO":
            raise ValueError(f"resume must be True, False or 'AUTO[+...]', got {resume!r}")
        rc = cls()
        for s in suffixes:
            table = {"ERRORED": ("resume", "resume"), "RESTART_ERRORED": ("resume", "restart"),
                     "ERRORED_ONLY": ("skip", "resume"), "RESTART_ERRORED_ONLY": ("skip", "restart")}
            if s not in table:
                raise ValueError(f"Invalid resume setting: {s!r}")
            rc = cls(unfinished=table[s][0], errored=table[s][1])
        return rc


# ------------------------------------------------------------------------- progress reporting
class ProgressReporter:
    """Base reporter: ``should_report`` gates ``report(trials, done)``; used as a Tuner callback."""

    def __init__(self, metric_columns: Optional[Union[List[str], Dict[str, str]]] = None,
                 parameter_columns: Optional[Union[List[str], Dict[str, str]]] = None,
                 max_report_frequency: float = 5.0, metric: Optional[str] = None, mode: Optional[str] = None,
                 max_progress_rows: int = 20, **kw):
        self.metric_columns = metric_columns
        self.parameter_columns = parameter_columns
        self.max_report_frequency = max_report_frequency
        self.metric, self.mode = metric, mode
        self.max_progress_rows = max_progress_rows
        self._last = 0.0
        self._trials: Dict[str, dict] = {}

    def add_metric_column(self, metric: str, representation: Optional[str] = None):
        if isinstance(self.metric_columns, dict):
            self.metric_columns[metric] = representation or metric
        else:
            self.metric_columns = list(self.metric_columns or []) + [metric]

    def should_report(self, trials, done: bool = False) -> bool:
        return done or time.time() - self._last >= self.max_report_frequency

    def report(self, trials, done: bool, *sys_info):
        raise NotImplementedError

    # Tuner callback hooks -------------------------------------------------------------
    def _row(self, trial, result, status):
        self._trials[getattr(trial, "trial_id", str(trial))] = {
            "trial_id": getattr(trial, "trial_id", str(trial)), "status": status,
            "config": dict(getattr(trial, "config", {}) or {}), "result": dict(result or {})}

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self._row(trial, result, "RUNNING")
        if self.should_report(trials):
            self._last = time.time()
            self.report(list(self._trials.values()), False)

    def on_trial_complete(self, iteration, trials, trial, **info):
        prev = self._trials.get(getattr(trial, "trial_id", str(trial)), {}).get("result")
        self._row(trial, prev, "TERMINATED")

    def on_experiment_end(self, trials, **info):
        self.report(list(self._trials.values()), True)

    # table rendering -------------------------------------------------------------------
    def _columns(self, rows):
        metrics = self.metric_columns
        if metrics is None:
            keys = []
            for r in rows:
                for k, v in r["result"].items():
                    if isinstance(v, (int, float)) and k not in keys and not k.startswith(("time_", "timestamp")):
                        keys.append(k)
            metrics = keys[:6]
        params = self.parameter_columns
        if params is None:
            params = sorted({k for r in rows for k in r["config"]})[:6]
        m = metrics if isinstance(metrics, dict) else {k: k for k in metrics}
        p = params if isinstance(params, dict) else {k: k for k in params}
        return p, m

    def _table(self, rows) -> str:
        p, m = self._columns(rows)
        head = ["Trial name", "status"] + list(p.values()) + list(m.values())
        body = []
        for r in rows[: self.max_progress_rows]:
            body.append([r["trial_id"], r["status"]] + [_fmt(r["config"].get(k)) for k in p] +
                        [_fmt(r["result"].get(k)) for k in m])
        w = [max(len(str(x)) for x in col) for col in zip(head, *body)] if body else [len(h) for h in head]
        line = lambda cells: "| " + " | ".join(str(c).ljust(n) for c, n in zip(cells, w)) + " |"  # noqa: E731
        sep = "+" + "+".join("-" * (n + 2) for n in w) + "+"
        counts: Dict[str, int] = {}
        for r in rows:
            counts[r["status"]] = counts.get(r["status"], 0) + 1
        status = "Number of trials: " + ", ".join(f"{v} {k}" for k, v in sorted(counts.items()))
        return "\n".join([status, sep, line(head), sep] + [line(b) for b in body] + [sep])


def _fmt(v):
    if isinstance(v, float):
        return f"{v:.5g}"
    return "" if v is None else v


class CLIReporter(ProgressReporter):
    def __init__(self, *a, out=None, **kw):
        super().__init__(*a, **kw)
        self._out = out

    def report(self, trials, done, *sys_info):
        out = self._out or sys.stdout
        print(("== Status ==" if not done else "== Final status =="), file=out)
        print(self._table(trials), file=out, flush=True)


class JupyterNotebookReporter(CLIReporter):
    """Same table; in a notebook the reference renders HTML, here it prints text."""
