"""Tune result loggers (reference: ``python/ray/tune/logger/``: ``logger.py`` LoggerCallback /
Logger, ``csv.py`` CSVLoggerCallback, ``json.py`` JsonLoggerCallback, ``tensorboardx.py``
TBXLoggerCallback).

Every trial directory gets ``params.json`` (the resolved config), ``progress.csv`` (one row per
reported result, flattened ``a/b`` keys, header fixed by the first result as in the reference) and
``result.json`` (one JSON line per result; the experiment controller writes it for every trial since
``Result.from_path`` / ``Tuner.restore`` read it). The CSV and JSON callbacks are added by default
unless ``TUNE_DISABLE_AUTO_CALLBACK_LOGGERS=1`` or the run config already holds one of that class;
``TBXLoggerCallback`` writes TensorBoard scalars through ``torch.utils.tensorboard`` when that
import works (the tensorboard package is optional) and otherwise raises at construction.
"""
from __future__ import annotations

import csv
import json
import os
from typing import Any, Dict, List

from .. import Callback

DEFAULT_LOGGERS = ("CSVLoggerCallback", "JsonLoggerCallback")
EXPR_PARAM_FILE = "params.json"
EXPR_PROGRESS_FILE = "progress.csv"
EXPR_RESULT_FILE = "result.json"


def _flatten(d: Dict[str, Any], prefix: str = "", sep: str = "/") -> Dict[str, Any]:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{sep}{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(_flatten(v, key, sep))
        else:
            out[key] = v
    return out


def _jsonable(v):
    try:
        json.dumps(v)
        return v
    except TypeError:
        if isinstance(v, dict):
            return {str(k): _jsonable(x) for k, x in v.items()}
        if isinstance(v, (list, tuple)):
            return [_jsonable(x) for x in v]
        return repr(v)


class Logger:
    """Legacy per-trial logger interface (``Logger(config, logdir, trial)``)."""

    def __init__(self, config: Dict, logdir: str, trial=None):
        self.config = config
        self.logdir = logdir
        self.trial = trial
        self._init()

    def _init(self):
        pass

    def on_result(self, result: Dict):
        raise NotImplementedError

    def update_config(self, config: Dict):
        pass

    def close(self):
        pass

    def flush(self):
        pass


class LoggerCallback(Callback):
    """Base class: override ``log_trial_start`` / ``log_trial_result`` / ``log_trial_end``."""

    def log_trial_start(self, trial):
        pass

    def log_trial_restore(self, trial):
        pass

    def log_trial_save(self, trial):
        pass

    def log_trial_result(self, iteration: int, trial, result: Dict):
        pass

    def log_trial_end(self, trial, failed: bool = False):
        pass

    # Callback hooks the experiment controller calls
    def on_trial_start(self, iteration, trials, trial, **info):
        self.log_trial_start(trial)

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self.log_trial_result(iteration, trial, result)

    def on_trial_complete(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=getattr(trial, "status", "") == "ERROR")

    def on_trial_error(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=True)


class LegacyLoggerCallback(LoggerCallback):
    """Drives ``Logger`` subclasses, one instance per trial per class."""

    def __init__(self, logger_classes):
        self.logger_classes = list(logger_classes)
        self._loggers: Dict[str, List[Logger]] = {}

    def log_trial_start(self, trial):
        if trial.trial_id not in self._loggers:
            self._loggers[trial.trial_id] = [c(trial.config, trial.local_path, trial) for c in self.logger_classes]

    def log_trial_result(self, iteration, trial, result):
        self.log_trial_start(trial)
        for lg in self._loggers[trial.trial_id]:
            lg.on_result(result)

    def log_trial_end(self, trial, failed=False):
        for lg in self._loggers.pop(trial.trial_id, []):
            lg.close()


class JsonLoggerCallback(LoggerCallback):
    """``params.json`` per trial (``result.json`` lines come from the controller, see module doc)."""

    def log_trial_start(self, trial):
        os.makedirs(trial.local_path, exist_ok=True)
        with open(os.path.join(trial.local_path, EXPR_PARAM_FILE), "w") as f:
            json.dump(_jsonable(trial.config), f, indent=2, sort_keys=True)


class CSVLoggerCallback(LoggerCallback):
    """``progress.csv`` per trial: flattened keys of the first result form the header; later
    results fill those columns (new keys are dropped, like the reference's CSV logger)."""

    def __init__(self):
        self._files: Dict[str, Any] = {}

    def _writer(self, trial, result):
        ent = self._files.get(trial.trial_id)
        if ent is None:
            os.makedirs(trial.local_path, exist_ok=True)
            path = os.path.join(trial.local_path, EXPR_PROGRESS_FILE)
            exists = os.path.exists(path) and os.path.getsize(path) > 0
            f = open(path, "a", newline="")
            if exists:  # restored trial: keep the original header
                with open(path) as r:
                    header = next(csv.reader(r))
            else:
                header = [k for k in _flatten(result) if k != "config" and not k.startswith("config/")]
            w = csv.DictWriter(f, header, extrasaction="ignore")
            if not exists:
                w.writeheader()
            ent = self._files[trial.trial_id] = (f, w)
        return ent

    def log_trial_result(self, iteration, trial, result):
        flat = {k: v for k, v in _flatten(result).items() if k != "config" and not k.startswith("config/")}
        f, w = self._writer(trial, flat)
        w.writerow(flat)
        f.flush()

    def log_trial_end(self, trial, failed=False):
        ent = self._files.pop(trial.trial_id, None)
        if ent is not None:
            ent[0].close()


class TBXLoggerCallback(LoggerCallback):
    """TensorBoard scalars of every numeric result key, step = ``training_iteration``."""

    def __init__(self):
        try:
            from torch.utils.tensorboard import SummaryWriter  # noqa: F401
        except Exception as e:  # tensorboard is not installed on this platform
            raise ImportError("TBXLoggerCallback needs torch.utils.tensorboard (the tensorboard package)") from e
        self._writers: Dict[str, Any] = {}

    def log_trial_result(self, iteration, trial, result):
        from torch.utils.tensorboard import SummaryWriter

        w = self._writers.get(trial.trial_id)
        if w is None:
            w = self._writers[trial.trial_id] = SummaryWriter(trial.local_path)
        step = int(result.get("training_iteration", iteration))
        for k, v in _flatten(result).items():
            if isinstance(v, (int, float)) and not isinstance(v, bool) and not k.startswith("config/"):
                w.add_scalar(f"ray/tune/{k}", v, global_step=step)
        w.flush()

    def log_trial_end(self, trial, failed=False):
        w = self._writers.pop(trial.trial_id, None)
        if w is not None:
            w.close()


class CSVLogger(Logger):
    def _init(self):
        self._cb = CSVLoggerCallback()

    def on_result(self, result):
        self._cb.log_trial_result(0, self.trial, result)

    def close(self):
        self._cb.log_trial_end(self.trial)


class JsonLogger(Logger):
    def _init(self):
        JsonLoggerCallback().log_trial_start(self.trial)

    def on_result(self, result):
        pass


def default_logger_callbacks(existing) -> list:
    """The CSV / JSON logger callbacks missing from ``existing`` (reference:
    ``tune/utils/callback.py`` ``_create_default_callbacks``)."""
    if os.environ.get("TUNE_DISABLE_AUTO_CALLBACK_LOGGERS", "0") == "1":
        return []
    have = {type(c) for c in existing or []}
    out = []
    if not any(issubclass(t, CSVLoggerCallback) for t in have):
        out.append(CSVLoggerCallback())
    if not any(issubclass(t, JsonLoggerCallback) for t in have):
        out.append(JsonLoggerCallback())
    return out


__all__ = ["Logger", "LoggerCallback", "LegacyLoggerCallback", "CSVLoggerCallback", "JsonLoggerCallback",
           "TBXLoggerCallback", "CSVLogger", "JsonLogger", "DEFAULT_LOGGERS", "default_logger_callbacks"]
