"""DataParallelTrainer / BaseTrainer (reference: ``python/ray/train/data_parallel_trainer.py``,
``python/ray/train/base_trainer.py``)."""
from __future__ import annotations

import inspect
import os
import time
import uuid
from typing import Any, Callable, Dict, Optional, Union

from ..air.config import RunConfig, ScalingConfig
from ..air.result import Result
from .backend import BackendConfig


from ._internal.backend_executor import TrainingFailedError


def _in_external_launcher() -> bool:
    """True when this process is one rank of an external SPMD launch (torchrun) rather than a
    framework-managed worker group."""
    env = os.environ
    if env.get("RCA_WORKER_ID"):
        return False
    return bool(env.get("TORCHELASTIC_RUN_ID")) or (int(env.get("WORLD_SIZE", "1")) > 1 and "RANK" in env)


class BaseTrainer:
    def __init__(self, *, scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 datasets: Optional[Dict[str, Any]] = None, resume_from_checkpoint=None,
                 metadata: Optional[Dict[str, Any]] = None):
        self.scaling_config = scaling_config or ScalingConfig(num_workers=1)
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.resume_from_checkpoint = resume_from_checkpoint
        self.metadata = metadata or {}

    def setup(self):
        pass

    def fit(self) -> Result:
        raise NotImplementedError

    def preprocess_datasets(self) -> None:
        """Deprecated in the reference (preprocessors are applied to datasets before passing them
        in); kept as a no-op hook that subclasses may still override."""

    def training_loop(self) -> None:
        """The trainer's main loop (reference: the method ``fit`` runs inside its Tune trial);
        here ``fit`` drives the worker group directly, so this runs it and keeps the result."""
        self._training_loop_result = self.fit()

    def as_trainable(self):
        trainer = self

        def trainable(config):
            t = trainer._with_config(config)
            return t._fit_in_trial()

        trainable._rca_trainer = trainer
        return trainable

    @classmethod
    def can_restore(cls, path) -> bool:
        return os.path.exists(os.path.join(path, "result.json"))

    @classmethod
    def restore(cls, path, **kwargs):
        r = Result.from_path(path)
        t = cls(**kwargs)
        t.resume_from_checkpoint = r.checkpoint
        return t


class DataParallelTrainer(BaseTrainer):
    _default_backend_config = BackendConfig()

    def get_dataset_config(self):
        """The ``DataConfig`` the datasets are split with (the default one if none was given)."""
        if self.dataset_config is not None:
            return self.dataset_config
        from . import DataConfig

        return DataConfig()

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[Dict] = None,
                 backend_config: Optional[BackendConfig] = None, scaling_config: Optional[ScalingConfig] = None,
                 run_config: Optional[RunConfig] = None, datasets: Optional[Dict[str, Any]] = None,
                 dataset_config=None, resume_from_checkpoint=None, metadata: Optional[Dict[str, Any]] = None):
        super().__init__(scaling_config=scaling_config, run_config=run_config, datasets=datasets,
                         resume_from_checkpoint=resume_from_checkpoint, metadata=metadata)
        self.train_loop_per_worker = train_loop_per_worker
        self.train_loop_config = train_loop_config
        self.backend_config = backend_config or self._default_backend_config
        self.dataset_config = dataset_config
        nparams = len(inspect.signature(train_loop_per_worker).parameters)
        if nparams > 1:
            raise ValueError(f"train_loop_per_worker should take 0 or 1 arguments, got {nparams}.")
        self._takes_config = nparams == 1

    def _with_config(self, config):
        import copy

        t = copy.copy(self)
        cfg = dict(self.train_loop_config or {})
        cfg.update(config.get("train_loop_config", config) if isinstance(config, dict) else {})
        t.train_loop_config = cfg
        return t

    def _experiment_dir(self):
        name = self.run_config.name or f"{type(self).__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        return name, os.path.join(os.path.expanduser(self.run_config.storage_path), name)

    def fit(self) -> Result:
        if _in_external_launcher():
            return self._fit_external()
        from .._private import worker as w

        if not w.is_initialized():
            w.init()
        name, exp_dir = self._experiment_dir()
        trial_dir = exp_dir
        result = self._run(trial_dir, name, self._standalone_reporter(trial_dir))
        cbs = list(getattr(self.run_config, "callbacks", None) or [])
        if cbs:
            trial = self._cb_trial
            trial.status = "ERROR" if result.error is not None else "TERMINATED"
            for cb in cbs:
                if hasattr(cb, "on_trial_complete"):
                    cb.on_trial_complete(iteration=0, trials=[trial], trial=trial)
        if result.error is not None and not getattr(self, "_in_tune", False):
            raise result.error
        return result

    def _standalone_reporter(self, trial_dir):
        """``fit()`` outside Tune still honours ``RunConfig.stop`` and ``RunConfig.callbacks`` (the
        reference runs every trainer through a one-trial Tune experiment)."""
        from ..tune.tuner import Trial, evaluate_stop

        stop = getattr(self.run_config, "stop", None)
        cbs = list(getattr(self.run_config, "callbacks", None) or [])
        trial = Trial(os.path.basename(trial_dir), dict(self.train_loop_config or {}), trial_dir, {})
        trial.status = "RUNNING"
        trial.start_time = time.time()
        self._cb_trial = trial
        if stop is None and not cbs:
            return None

        def on_report(metrics, checkpoint):
            trial.last_result = metrics
            trial.metrics_history.append(metrics)
            if checkpoint is not None:
                trial.checkpoint = checkpoint
            for cb in cbs:
                if hasattr(cb, "on_trial_result"):
                    cb.on_trial_result(iteration=len(trial.metrics_history), trials=[trial], trial=trial,
                                       result=metrics)
            s, s_all = evaluate_stop(stop, trial.trial_id, metrics)
            return s or s_all

        return on_report

    def _fit_in_trial(self, trial_dir=None, report_callback=None):
        name, exp_dir = self._experiment_dir()
        return self._run(trial_dir or exp_dir, name, report_callback)

    def _run(self, trial_dir, name, report_callback=None):
        from ._internal.backend_executor import run_training

        backend = self.backend_config.backend_cls()
        cfg = self.train_loop_config if self._takes_config else None
        fn = self.train_loop_per_worker
        if self._takes_config and cfg is None:
            cfg = {}
        return run_training(fn, cfg, self.scaling_config, self.run_config, backend, self.backend_config,
                            self.datasets, self.dataset_config, self.resume_from_checkpoint, trial_dir,
                            metadata=self.metadata, report_callback=report_callback, experiment_name=name)

    # -------------------------------------------------------------- torchrun / SPMD mode
    def _fit_external(self) -> Result:
        """Run this rank's share of the job in-process (external launcher owns the processes)."""
        from ._internal import session as S

        self._setup_external_backend()
        S.shutdown_session()
        sess = S.get_session()
        sess.checkpoint = self.resume_from_checkpoint
        if self.datasets:
            ctx = sess.context
            for k, ds in self.datasets.items():
                if hasattr(ds, "split"):
                    sess.dataset_shards[k] = ds.split(ctx.world_size, equal=True)[ctx.world_rank].iterator()
                else:
                    sess.dataset_shards[k] = ds
        err = None
        try:
            if self._takes_config:
                self.train_loop_per_worker(dict(self.train_loop_config or {}))
            else:
                self.train_loop_per_worker()
        except BaseException as e:  # noqa
            err = TrainingFailedError(f"Training failed: {e}")
            err.__cause__ = e
        hist = sess.history
        r = Result(metrics=hist[-1] if hist else None, checkpoint=sess.checkpoint, error=err, path=None,
                   metrics_history=hist)
        if err is not None:
            raise err
        return r

    def _setup_external_backend(self):
        pass
