"""Ray Tune equivalent (reference: ``python/ray/tune``)."""
from __future__ import annotations

import functools
import inspect
from typing import Any, Callable, Dict, Optional

from ..air.config import CheckpointConfig, FailureConfig, RunConfig, SyncConfig
from ..air.result import Result
from ..train._checkpoint import Checkpoint
from .schedulers import (ASHAScheduler, AsyncHyperBandScheduler, FIFOScheduler, HyperBandScheduler,
                         MedianStoppingRule, PopulationBasedTraining, TrialScheduler)
from .search import BasicVariantGenerator, ConcurrencyLimiter, Searcher
from .search.sample import (choice, grid_search, lograndint, loguniform, qlograndint, qloguniform, qrandint, qrandn,
                            quniform, randint, randn, sample_from, uniform)
from .tuner import ResultGrid, Stopper, Trainable, TuneConfig, Tuner
from .registry import (CLIReporter, Experiment, JupyterNotebookReporter, PlacementGroupFactory, ProgressReporter,
                       ResumeConfig, create_scheduler, create_searcher, register_env, register_trainable,
                       run_experiments)


def report(metrics: Optional[Dict] = None, *, checkpoint=None, **kwargs):
    """Report from a function trainable (``tune.report(metrics)`` or legacy ``tune.report(a=1)``)."""
    from ..train import report as _report

    m = dict(metrics or {})
    m.update(kwargs)
    _report(m, checkpoint=checkpoint)


def get_checkpoint():
    from ..train import get_checkpoint as _g

    return _g()


def get_context():
    from ..train import get_context as _g

    return _g()


def with_resources(trainable, resources):
    if isinstance(resources, PlacementGroupFactory):
        resources = resources.required_resources
    if callable(resources) and not isinstance(resources, dict):
        raise NotImplementedError("resource functions are not supported; pass a dict")
    res = {}
    for k, v in dict(resources).items():
        res[{"cpu": "CPU", "gpu": "GPU"}.get(k, k)] = v
    if inspect.isclass(trainable):
        trainable._rca_resources = res
        return trainable

    @functools.wraps(trainable)
    def wrapped(*a, **k):
        return trainable(*a, **k)

    wrapped._rca_resources = res
    return wrapped


def with_parameters(trainable, **kwargs):
    """Put large parameters in the object store once; every trial fetches them by reference."""
    from .._private.worker import get, put

    refs = {k: put(v) for k, v in kwargs.items()}

    if inspect.isclass(trainable):
        class _Wrapped(trainable):
            def setup(self, config):
                extra = {k: get(r) for k, r in refs.items()}
                super().setup(config, **extra)

        _Wrapped.__name__ = trainable.__name__
        return _Wrapped

    def wrapped(config):
        extra = {k: get(r) for k, r in refs.items()}
        return trainable(config, **extra)

    wrapped.__name__ = getattr(trainable, "__name__", "trainable")
    if hasattr(trainable, "_rca_resources"):
        wrapped._rca_resources = trainable._rca_resources
    return wrapped


def run(run_or_experiment, *, name=None, metric=None, mode=None, stop=None, config=None, resources_per_trial=None,
        num_samples=1, storage_path=None, search_alg=None, scheduler=None, checkpoint_config=None,
        max_failures=0, max_concurrent_trials=None, time_budget_s=None, callbacks=None, verbose=None,
        fail_fast=False, raise_on_failed_trial=True, progress_reporter=None, **kwargs) -> "ExperimentAnalysis":
    """Legacy functional API: returns an ExperimentAnalysis."""
    from .registry import resolve_trainable

    t = resolve_trainable(run_or_experiment)
    if progress_reporter is not None:
        callbacks = list(callbacks or []) + [progress_reporter]
    if resources_per_trial:
        t = with_resources(t, resources_per_trial)
    tuner = Tuner(t, param_space=config or {},
                  tune_config=TuneConfig(metric=metric, mode=mode, num_samples=num_samples, search_alg=search_alg,
                                         scheduler=scheduler, max_concurrent_trials=max_concurrent_trials,
                                         time_budget_s=time_budget_s),
                  run_config=RunConfig(name=name, storage_path=storage_path, stop=stop, callbacks=callbacks,
                                       checkpoint_config=checkpoint_config or CheckpointConfig(),
                                       failure_config=FailureConfig(max_failures=max_failures, fail_fast=fail_fast)))
    grid = tuner.fit()
    if raise_on_failed_trial and grid.num_errors:
        raise TuneError(f"Trials did not complete: {grid.errors}")
    return ExperimentAnalysis(grid, metric, mode)


class TuneError(Exception):
    pass


class ExperimentAnalysis:
    def __init__(self, grid: ResultGrid, metric=None, mode=None):
        self._grid = grid
        self.default_metric = metric
        self.default_mode = mode

    @property
    def trials(self):
        return list(self._grid)

    def get_best_config(self, metric=None, mode=None, scope="last"):
        return self._grid.get_best_result(metric or self.default_metric, mode or self.default_mode, scope).config

    @property
    def best_config(self):
        return self.get_best_config()

    @property
    def best_result(self):
        return self._grid.get_best_result(self.default_metric, self.default_mode).metrics

    @property
    def best_checkpoint(self):
        return self._grid.get_best_result(self.default_metric, self.default_mode).checkpoint

    @property
    def results_df(self):
        return self._grid.get_dataframe()

    def dataframe(self, metric=None, mode=None):
        return self._grid.get_dataframe()


class Callback:
    def on_trial_result(self, iteration, trials, trial, result, **info):
        pass

    def on_trial_complete(self, iteration, trials, trial, **info):
        pass


__all__ = ["SyncConfig", "Tuner", "TuneConfig", "ResultGrid", "Trainable", "Stopper", "report", "get_checkpoint", "get_context",
           "run", "with_resources", "with_parameters", "choice", "uniform", "quniform", "loguniform", "qloguniform",
           "randn", "qrandn", "randint", "qrandint", "lograndint", "qlograndint", "sample_from", "grid_search",
           "ASHAScheduler", "AsyncHyperBandScheduler", "HyperBandScheduler", "MedianStoppingRule",
           "PopulationBasedTraining", "FIFOScheduler", "TrialScheduler", "BasicVariantGenerator",
           "ConcurrencyLimiter", "Searcher", "Checkpoint", "RunConfig", "CheckpointConfig", "FailureConfig",
           "Result", "Callback", "ExperimentAnalysis", "TuneError", "register_env", "register_trainable",
           "run_experiments", "Experiment", "CLIReporter", "JupyterNotebookReporter", "ProgressReporter",
           "create_searcher", "create_scheduler", "PlacementGroupFactory", "ResumeConfig"]
