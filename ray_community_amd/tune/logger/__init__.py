"""Tune result loggers (reference: ``python/ray/tune/logger/``: ``logger.py`` LoggerCallback /
Logger, ``csv.py`` CSVLoggerCallback, ``json.py`` JsonLoggerCallback, ``tensorboardx.py``
TBXLoggerCallback).

Every trial directory gets ``params.json`` (the resolved config), ``progress.csv`` (one row per
reported result, flattened ``a/b`` keys, header fixed by the first result as in the reference) and
``result.json`` (one JSON line per result; the experiment controller writes it for every trial since
``Result.from_path`` / ``Tuner.restore`` read it). The CSV and JSON callbacks are added by default
unless ``TUNE_DISABLE_AUTO_CALLBACK_LOGGERS=1`` or the run config already holds one of that class;
``TBXLoggerCallback`` writes TensorBoard scalars as tfevents files with a built-in protobuf /
TFRecord encoder (tensorboard itself is not installed here).
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


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _scalar_event(wall_time: float, step: int, tag: str, value: float) -> bytes:
    """tensorboard ``Event{wall_time, step, summary{value{tag, simple_value}}}`` in protobuf wire
    format (event.proto / summary.proto field numbers), encoded by hand: no tensorboard needed."""
    import struct

    t = tag.encode()
    val = _field(1, 2, _varint(len(t)) + t) + _field(2, 5, struct.pack("<f", float(value)))
    summ = _field(1, 2, _varint(len(val)) + val)
    return (_field(1, 1, struct.pack("<d", wall_time)) + _field(2, 0, _varint(int(step)))
            + _field(5, 2, _varint(len(summ)) + summ))


class _EventFile:
    """Append-only ``events.out.tfevents.*`` writer: TFRecord framing (length, masked CRC32C of the
    length, payload, masked CRC32C of the payload) around Event protos."""

    def __init__(self, logdir: str):
        import socket
        import struct
        import time

        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self._f = open(self.path, "ab")
        ver = b"brain.Event:2"
        self._write(_field(1, 1, struct.pack("<d", time.time())) + _field(3, 2, _varint(len(ver)) + ver))

    def _write(self, payload: bytes):
        import struct

        from ...data.datasource import _masked_crc

        hdr = struct.pack("<Q", len(payload))
        self._f.write(hdr + struct.pack("<I", _masked_crc(hdr)) + payload + struct.pack("<I", _masked_crc(payload)))

    def add_scalar(self, tag: str, value: float, step: int):
        import time

        self._write(_scalar_event(time.time(), step, tag, value))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


class TBXLoggerCallback(LoggerCallback):
    """TensorBoard scalars (``ray/tune/<key>``) of every numeric result key, step =
    ``training_iteration``, written as tfevents files in each trial directory by a built-in
    encoder (the tensorboard / tensorboardX packages are not needed)."""

    def __init__(self):
        self._writers: Dict[str, _EventFile] = {}

    def log_trial_result(self, iteration, trial, result):
        w = self._writers.get(trial.trial_id)
        if w is None:
            w = self._writers[trial.trial_id] = _EventFile(trial.local_path)
        step = int(result.get("training_iteration", iteration))
        for k, v in _flatten(result).items():
            if isinstance(v, (int, float)) and not isinstance(v, bool) and not k.startswith("config/"):
                w.add_scalar(f"ray/tune/{k}", v, step)
        w.flush()

    def log_trial_end(self, trial, failed=False):
        w = self._writers.pop(trial.trial_id, None)
        if w is not None:
            w.close()


class _LogTarget:
    """What the logger callbacks read from a trial, for a ``Logger`` built as
    ``Logger(config, logdir)`` without one."""

    def __init__(self, config, logdir, trial):
        self.trial_id = getattr(trial, "trial_id", None) or logdir
        self.local_path = getattr(trial, "local_path", None) or logdir
        self.config = config


class CSVLogger(Logger):
    def _init(self):
        self._cb = CSVLoggerCallback()
        self._t = _LogTarget(self.config, self.logdir, self.trial)

    def on_result(self, result):
        self._cb.log_trial_result(0, self._t, result)

    def close(self):
        self._cb.log_trial_end(self._t)


class JsonLogger(Logger):
    def _init(self):
        JsonLoggerCallback().log_trial_start(_LogTarget(self.config, self.logdir, self.trial))

    def on_result(self, result):
        pass

    def update_config(self, config):
        self.config = config
        JsonLoggerCallback().log_trial_start(_LogTarget(config, self.logdir, self.trial))


class TBXLogger(Logger):
    """TensorBoard scalars for one trial (reference tune/logger/tensorboardx.py)."""

    def _init(self):
        self._cb = TBXLoggerCallback()
        self._t = _LogTarget(self.config, self.logdir, self.trial)

    def on_result(self, result):
        self._cb.log_trial_result(0, self._t, result)

    def close(self):
        self._cb.log_trial_end(self._t)


class NoopLogger(Logger):
    def on_result(self, result):
        pass


class UnifiedLogger(Logger):
    """Fans results out to ``loggers`` (default JSON, CSV and TensorBoard), reference
    tune/logger/unified.py."""

    def __init__(self, config: Dict, logdir: str, trial=None, loggers=None):
        self._logger_cls_list = list(loggers) if loggers is not None else [JsonLogger, CSVLogger, TBXLogger]
        super().__init__(config, logdir, trial)

    def _init(self):
        self._loggers = [cls(self.config, self.logdir, self.trial) for cls in self._logger_cls_list]

    def on_result(self, result):
        for lg in self._loggers:
            lg.on_result(result)

    def update_config(self, config):
        for lg in self._loggers:
            lg.update_config(config)

    def close(self):
        for lg in self._loggers:
            lg.close()

    def flush(self):
        for lg in self._loggers:
            lg.flush()


def pretty_print(result: Dict, exclude=None) -> str:
    """A result dict as YAML without ``config`` / ``hist_stats`` (and ``exclude`` keys), values
    that JSON cannot hold shown as their repr (reference tune/logger/logger.py:pretty_print)."""
    import yaml

    out = {k: v for k, v in result.items()
           if v is not None and k not in ("config", "hist_stats") and (exclude is None or k not in exclude)}
    return yaml.safe_dump(json.loads(json.dumps(_jsonable(out))), default_flow_style=False)


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
           "TBXLoggerCallback", "CSVLogger", "JsonLogger", "TBXLogger", "NoopLogger", "UnifiedLogger", "pretty_print",
           "DEFAULT_LOGGERS", "default_logger_callbacks"]
