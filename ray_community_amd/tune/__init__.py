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
from .analysis import ExperimentAnalysis
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
        fail_fast=False, raise_on_failed_trial=True, progress_reporter=None, storage_filesystem=None,
        log_to_file=False, trial_name_creator=None, trial_dirname_creator=None, sync_config=None,
        export_formats=None, restore=None, resume=None, resume_config=None, reuse_actors=False,
        keep_checkpoints_num=None, checkpoint_score_attr=None, checkpoint_freq=0, checkpoint_at_end=False,
        chdir_to_trial_dir=None, local_dir=None, **kwargs) -> "ExperimentAnalysis":
    """Legacy functional API: returns an ExperimentAnalysis (reference: python/ray/tune/tune.py:277).

    The pre-2.7 keyword arguments map onto the Tuner's configs: ``local_dir`` is ``storage_path``;
    ``keep_checkpoints_num`` / ``checkpoint_score_attr`` ("min-<metric>" for ascending) /
    ``checkpoint_freq`` / ``checkpoint_at_end`` fill the CheckpointConfig; ``resume`` (True, "AUTO",
    "AUTO+ERRORED", ...) or ``resume_config`` restores the experiment at ``storage_path/name``
    through ``Tuner.restore``; ``restore`` seeds every trial from one checkpoint directory."""
    import os

    from .registry import ResumeConfig, resolve_trainable

    if kwargs:
        raise TypeError(f"tune.run() got unexpected keyword arguments: {sorted(kwargs)}")
    if local_dir is not None:
        if storage_path is not None and storage_path != local_dir:
            raise ValueError("Pass only one of storage_path and local_dir (its pre-2.7 name)")
        storage_path = local_dir
    t = resolve_trainable(run_or_experiment)
    if progress_reporter is not None:
        callbacks = list(callbacks or []) + [progress_reporter]
    if resources_per_trial:
        t = with_resources(t, resources_per_trial)
    ckpt = checkpoint_config or CheckpointConfig()
    if keep_checkpoints_num is not None:
        ckpt.num_to_keep = keep_checkpoints_num
    if checkpoint_score_attr is not None:
        order, attr = ("min", checkpoint_score_attr[4:]) if checkpoint_score_attr.startswith("min-") \
            else ("max", checkpoint_score_attr)
        ckpt.checkpoint_score_attribute, ckpt.checkpoint_score_order = attr, order
    if checkpoint_freq:
        ckpt.checkpoint_frequency = checkpoint_freq
    if checkpoint_at_end:
        ckpt.checkpoint_at_end = True
    restore_dir = None
    if restore is not None:  # every trial starts from this checkpoint directory
        restore_dir = os.path.expanduser(restore)
        if not os.path.isdir(restore_dir):
            raise ValueError(f"restore={restore!r} is not a checkpoint directory")
    tc = TuneConfig(metric=metric, mode=mode, num_samples=num_samples, search_alg=search_alg,
                    scheduler=scheduler, max_concurrent_trials=max_concurrent_trials,
                    time_budget_s=time_budget_s, reuse_actors=reuse_actors,
                    trial_name_creator=trial_name_creator, trial_dirname_creator=trial_dirname_creator)
    rc = RunConfig(name=name, storage_path=storage_path, storage_filesystem=storage_filesystem, stop=stop,
                   callbacks=callbacks, checkpoint_config=ckpt, sync_config=sync_config, verbose=verbose,
                   log_to_file=log_to_file,
                   failure_config=FailureConfig(max_failures=max_failures, fail_fast=fail_fast))
    resume_config = resume_config or ResumeConfig._from_legacy(resume)
    tuner = None
    if resume_config is not None:
        if not name:
            raise ValueError("resume needs the experiment's name (tune.run(..., name=...))")
        exp_dir = os.path.join(os.path.expanduser(rc.storage_path), name)
        if Tuner.can_restore(exp_dir):
            tuner = Tuner.restore(exp_dir, t, param_space=config or {}, tune_config=tc, run_config=rc,
                                  **resume_config._restore_kwargs())
        elif resume is True:
            raise ValueError(f"resume=True but there is no experiment state under {exp_dir}")
    if tuner is None:  # a fresh run ("AUTO" with nothing to resume lands here too)
        tuner = Tuner(t, param_space=config or {}, tune_config=tc, run_config=rc)
        tuner._initial_restore = restore_dir
    grid = tuner.fit()
    if raise_on_failed_trial and grid.num_errors:
        raise TuneError(f"Trials did not complete: {grid.errors}")
    return ExperimentAnalysis(grid, default_metric=metric, default_mode=mode)


class TuneError(Exception):
    pass


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
