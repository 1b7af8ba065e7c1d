"""Tuner / trial controller / ResultGrid (reference: ``python/ray/tune/tuner.py``,
``tune/execution/tune_controller.py``, ``tune/result_grid.py``, ``tune/trainable/trainable.py``).

Trials run as actors (function and class trainables) or as driver-side threads that orchestrate
their own worker group (Train ``Trainer`` objects); the controller streams their reports,
applies stopping criteria, the scheduler's decisions and the searcher's suggestions, and keeps a
JSON experiment state so an interrupted experiment can be restored.
"""
from __future__ import annotations

import copy
import inspect
import json
import logging
import os
import queue
import shutil
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Union

from ..air.config import CheckpointConfig, FailureConfig, RunConfig
from ..air.result import Result
from .schedulers import FIFOScheduler, TrialScheduler
from .search import BasicVariantGenerator, ConcurrencyLimiter, Searcher

log = logging.getLogger("ray_community_amd.tune")

PENDING, RUNNING, PAUSED, TERMINATED, ERROR = "PENDING", "RUNNING", "PAUSED", "TERMINATED", "ERROR"


@dataclass
class TuneConfig:
    metric: Optional[str] = None
    mode: Optional[str] = None
    search_alg: Optional[Searcher] = None
    scheduler: Optional[TrialScheduler] = None
    num_samples: int = 1
    max_concurrent_trials: Optional[int] = None
    time_budget_s: Optional[float] = None
    reuse_actors: bool = False
    trial_name_creator: Optional[Callable] = None
    trial_dirname_creator: Optional[Callable] = None
    chdir_to_trial_dir: bool = False

    def __post_init__(self):
        if self.mode not in (None, "min", "max"):
            raise ValueError("`mode` must be 'min' or 'max'")


class Trainable:
    """Class API: override setup/step/save_checkpoint/load_checkpoint."""

    def __init__(self, config: Optional[Dict] = None, **kw):
        self.config = config or {}
        self._iteration = 0
        # trial identity (set by the trial runner before construction, so setup() can see it)
        self._trial_info = dict(kw.get("trial_info") or _CURRENT_TRIAL_INFO)
        self.setup(copy.deepcopy(self.config))

    @property
    def trial_id(self) -> str:
        return self._info().get("trial_id", "default")

    @property
    def trial_name(self) -> str:
        return self._info().get("trial_name", "default")

    @property
    def logdir(self) -> Optional[str]:
        return self._info().get("logdir")

    def _info(self):
        return getattr(self, "_trial_info", None) or _CURRENT_TRIAL_INFO

    def setup(self, config):
        pass

    def step(self) -> Dict:
        raise NotImplementedError

    def save_checkpoint(self, checkpoint_dir: str) -> Optional[Dict]:
        return None

    def load_checkpoint(self, checkpoint):
        pass

    def cleanup(self):
        pass

    def reset_config(self, new_config) -> bool:
        return False

    @property
    def iteration(self):
        return self._iteration

    @property
    def training_iteration(self):
        return self._iteration

    # ------------------------------------------------------------------ direct-use API
    # (reference python/ray/tune/trainable/trainable.py: a class trainable can also be driven by
    # hand -- train / save / restore / reset / stop -- outside a Tuner)
    def get_config(self) -> Dict:
        return self.config

    def get_current_ip_pid(self):
        from ..util import get_node_ip_address

        return get_node_ip_address(), os.getpid()

    def is_actor(self) -> bool:
        return bool(os.environ.get("RCA_WORKER_ID"))

    @property
    def trial_resources(self):
        return self._info().get("resources")

    @classmethod
    def default_resource_request(cls, config):
        return None

    @classmethod
    def resource_help(cls, config) -> str:
        return ""

    def get_auto_filled_metrics(self, now=None, time_this_iter=None, timestamp=None, debug_metrics_only=False) -> Dict:
        out = {"training_iteration": self._iteration, "trial_id": self.trial_id}
        if not debug_metrics_only:
            out.update({"time_this_iter_s": time_this_iter, "timestamp": int(timestamp or time.time()),
                        "time_total_s": getattr(self, "_time_total", 0.0), "pid": os.getpid()})
        return out

    def log_result(self, result: Dict) -> None:
        self._last_result = dict(result)

    def train(self) -> Dict:
        """One ``step()`` with the auto-filled fields (training_iteration, timings, done)."""
        t0 = time.time()
        result = self.step()
        if not isinstance(result, dict):
            raise ValueError(f"step() must return a dict, got {type(result).__name__}")
        dt = time.time() - t0
        self._iteration += 1
        self._time_total = getattr(self, "_time_total", 0.0) + dt
        result = dict(result)
        result.setdefault("done", False)
        result.update(self.get_auto_filled_metrics(time_this_iter=dt))
        self.log_result(result)
        return result

    def train_buffered(self, buffer_time_s: float, max_buffer_length: int = 1000) -> List[Dict]:
        out, t0 = [], time.time()
        while len(out) < max_buffer_length and (not out or time.time() - t0 < buffer_time_s):
            r = self.train()
            out.append(r)
            if r.get("done"):
                break
        return out

    def get_state(self) -> Dict:
        return {"iteration": self._iteration, "time_total": getattr(self, "_time_total", 0.0),
                "config": self.config}

    def save(self, checkpoint_dir: Optional[str] = None):
        """``save_checkpoint`` into ``checkpoint_dir`` (a fresh temp dir by default); a returned dict
        is stored next to the files. Returns the checkpoint."""
        import pickle
        import tempfile

        from ..train._checkpoint import Checkpoint

        d = checkpoint_dir or tempfile.mkdtemp(prefix=f"checkpoint_{self._iteration:06d}_")
        os.makedirs(d, exist_ok=True)
        state = self.save_checkpoint(d)
        if isinstance(state, dict):
            with open(os.path.join(d, "_rca_trainable_state.pkl"), "wb") as f:
                pickle.dump(state, f)
        with open(os.path.join(d, "_rca_trainable_meta.json"), "w") as f:
            json.dump({"iteration": self._iteration, "time_total": getattr(self, "_time_total", 0.0)}, f)
        return Checkpoint.from_directory(d)

    def restore(self, checkpoint_path):
        """Inverse of ``save``: ``load_checkpoint`` gets the saved dict (or the directory) and the
        iteration counter is restored."""
        import pickle

        d = checkpoint_path if isinstance(checkpoint_path, str) else getattr(checkpoint_path, "path", checkpoint_path)
        meta = os.path.join(d, "_rca_trainable_meta.json")
        if os.path.exists(meta):
            with open(meta) as f:
                m = json.load(f)
            self._iteration, self._time_total = int(m["iteration"]), float(m["time_total"])
        st = os.path.join(d, "_rca_trainable_state.pkl")
        if os.path.exists(st):
            with open(st, "rb") as f:  # written by save() above, in this framework
                self.load_checkpoint(pickle.load(f))
        else:
            self.load_checkpoint(d)

    def reset(self, new_config, logger_creator=None, storage=None) -> bool:
        """Reuse this instance for a new config (``reset_config``); counters restart."""
        ok = self.reset_config(new_config)
        if ok:
            self.config = new_config
            self._iteration = 0
            self._time_total = 0.0
        return ok

    def stop(self) -> None:
        self.cleanup()

    def export_model(self, export_formats, export_dir: Optional[str] = None):
        if isinstance(export_formats, str):
            export_formats = [export_formats]
        export_dir = export_dir or self.logdir or "."
        return self._export_model(export_formats, export_dir)

    def _export_model(self, export_formats, export_dir):
        return {}


class Stopper:
    def __call__(self, trial_id: str, result: Dict) -> bool:
        return False

    def stop_all(self) -> bool:
        return False


_CURRENT_TRIAL_INFO: Dict = {}


class _ClassTrainableRunner:
    def __init__(self, cls, config, checkpoint_path=None, trial_info=None, log_paths=None):
        global _CURRENT_TRIAL_INFO
        if log_paths:  # RunConfig(log_to_file=...): this actor process is the trial's for its lifetime
            _redirect_fds(*log_paths)
        _CURRENT_TRIAL_INFO = dict(trial_info or {})
        self.t = cls(config)
        if checkpoint_path:
            st = None
            p = os.path.join(checkpoint_path, "_state.json")
            if os.path.exists(p):
                with open(p) as f:
                    st = json.load(f)
            if st:
                self.t._iteration = st.get("iteration", 0)
            data = self._load_dict(checkpoint_path)
            self.t.load_checkpoint(data if data is not None else checkpoint_path)

    @staticmethod
    def _load_dict(path):
        p = os.path.join(path, "_dict_checkpoint.pkl")
        if os.path.exists(p):
            import pickle

            with open(p, "rb") as f:
                return pickle.load(f)
        return None

    def reset(self, config, checkpoint_path=None, trial_info=None, log_paths=None) -> bool:
        """``reuse_actors``: take a new trial in this actor if the trainable's ``reset_config``
        accepts its config (reference ``Trainable.reset``)."""
        global _CURRENT_TRIAL_INFO
        if not self.t.reset_config(config):
            return False
        if log_paths:
            _redirect_fds(*log_paths)
        _CURRENT_TRIAL_INFO = dict(trial_info or {})
        self.t.config = config
        self.t._iteration = 0
        if checkpoint_path:
            p = os.path.join(checkpoint_path, "_state.json")
            if os.path.exists(p):
                with open(p) as f:
                    self.t._iteration = json.load(f).get("iteration", 0)
            data = self._load_dict(checkpoint_path)
            self.t.load_checkpoint(data if data is not None else checkpoint_path)
        return True

    def step(self):
        before = self.t._iteration
        r = self.t.step() or {}
        if self.t._iteration == before:  # trainables like Algorithm count their own iterations
            self.t._iteration += 1
        r = dict(r)
        r.setdefault("training_iteration", self.t._iteration)
        return r

    def save(self, path):
        os.makedirs(path, exist_ok=True)
        d = self.t.save_checkpoint(path)
        if isinstance(d, dict):
            import pickle

            with open(os.path.join(path, "_dict_checkpoint.pkl"), "wb") as f:
                pickle.dump(d, f)
        with open(os.path.join(path, "_state.json"), "w") as f:
            json.dump({"iteration": self.t._iteration}, f)
        return path

    def stop(self):
        self.t.cleanup()
        return True


def _add_flat_keys(m: Dict, prefix: str = "", out: Optional[Dict] = None):
    """Nested result dicts also get ``"outer/inner"`` keys (reference: metrics such as
    ``"env_runners/episode_return_mean"`` work in TuneConfig(metric=), stoppers, schedulers,
    searchers and ``get_best_result``); the nested values stay as they are."""
    out = m if out is None else out
    for k, v in list(m.items()):
        if isinstance(v, dict) and k != "config" and v:
            for k2, v2 in v.items():
                key = f"{prefix}{k}/{k2}"
                if isinstance(v2, dict):
                    _add_flat_keys({k2: v2}, prefix=f"{prefix}{k}/", out=out)
                else:
                    out.setdefault(key, v2)
    return out


def _result_value(result: Dict, key: str):
    """``result[key]``; a ``"a/b"`` key walks nested dicts (the reference flattens results with
    "/"), and RLlib's old ``sampler_results/<m>`` prefix falls back to the top-level ``<m>``."""
    if key in result:
        return result[key]
    if "/" not in key:
        return None
    node = result
    for part in key.split("/"):
        if not isinstance(node, dict) or part not in node:
            node = None
            break
        node = node[part]
    if node is None and key.startswith("sampler_results/"):
        node = result.get(key.split("/", 1)[1])
    return None if isinstance(node, dict) else node


def evaluate_stop(stop, trial_id, result):
    """``RunConfig.stop`` semantics (reference ``tune/stopper``): a dict stops once any listed
    metric reaches its value, a ``Stopper`` / callable decides per result (a Stopper's
    ``stop_all()`` ends the whole experiment), ``result["done"]`` always stops.
    Returns ``(stop_this_trial, stop_all)``."""
    if stop is None:
        return bool(result.get("done")), False
    if isinstance(stop, dict):
        for k, v in stop.items():
            got = _result_value(result, k)
            if got is not None and got >= v:
                return True, False
        return bool(result.get("done")), False
    if isinstance(stop, Stopper):
        return bool(stop(trial_id, result)), bool(stop.stop_all())
    if callable(stop):
        return bool(stop(trial_id, result)), False
    return False, False


class Trial:
    def __init__(self, trial_id: str, config: Dict, local_path: str, resources: Dict):
        self.trial_id = trial_id
        self.config = config
        self.local_path = local_path
        self.resources = resources
        self.status = PENDING
        self.last_result: Dict = {}
        self.metrics_history: List[Dict] = []
        self.checkpoint = None
        self.error: Optional[BaseException] = None
        self.num_failures = 0
        self.start_time = None
        self.runner = None
        self.thread_q: Optional[queue.Queue] = None
        self.stop_flag = False
        self.restore_path = None
        self.iteration_offset = 0

    def __repr__(self):
        return f"Trial({self.trial_id}, {self.status})"

    def __str__(self):
        return getattr(self, "trial_name", None) or self.trial_id

    # --------------------------------------------------------------- the reference Trial's read API
    # (python/ray/tune/experiment/trial.py: what callbacks, schedulers and stoppers read)
    @property
    def path(self) -> str:
        return self.local_path

    logdir = path

    @property
    def local_dir(self) -> str:
        return os.path.dirname(self.local_path)

    @property
    def experiment_dir_name(self) -> str:
        return os.path.basename(os.path.dirname(self.local_path))

    local_experiment_path = local_dir
    remote_experiment_path = local_dir

    @property
    def experiment_tag(self) -> str:
        return getattr(self, "_experiment_tag", "") or ",".join(f"{k}={v}" for k, v in _flat_cfg(self.config))

    def set_experiment_tag(self, tag: str) -> None:
        self._experiment_tag = tag

    @property
    def has_reported_at_least_once(self) -> bool:
        return bool(self.last_result)

    @property
    def node_ip(self) -> str:
        from ..util import get_node_ip_address

        return get_node_ip_address()

    def get_ray_actor_ip(self) -> Optional[str]:
        return self.node_ip if self.runner is not None else None

    @property
    def placement_group_factory(self):
        from .registry import PlacementGroupFactory

        return PlacementGroupFactory([dict(self.resources)])

    def create_placement_group_factory(self):
        return self.placement_group_factory

    def update_resources(self, resources: Dict) -> None:
        self.resources = dict(getattr(resources, "required_resources", resources))

    def set_status(self, status: str) -> None:
        self.status = status

    def set_config(self, config: Dict) -> None:
        self.config = config

    def update_last_result(self, result: Dict) -> None:
        self.last_result = result
        self.metrics_history.append(result)

    @property
    def metric_analysis(self) -> Dict[str, Dict[str, float]]:
        """Per numeric metric: max / min / avg / last over the reported results."""
        out: Dict[str, Dict[str, float]] = {}
        for r in self.metrics_history:
            for k, v in r.items():
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    d = out.setdefault(k, {"max": v, "min": v, "sum": 0.0, "n": 0})
                    d["max"], d["min"] = max(d["max"], v), min(d["min"], v)
                    d["sum"] += v
                    d["n"] += 1
                    d["last"] = v
        return {k: {"max": d["max"], "min": d["min"], "avg": d["sum"] / d["n"], "last": d["last"]}
                for k, d in out.items()}

    def is_finished(self) -> bool:
        return self.status in (TERMINATED, ERROR)

    def has_checkpoint(self) -> bool:
        return self.checkpoint is not None

    def clear_checkpoint(self) -> None:
        self.checkpoint = None

    @property
    def latest_checkpoint_result(self) -> Optional[Dict]:
        return self.last_result if self.checkpoint is not None else None

    def get_error(self) -> Optional[BaseException]:
        return self.error

    @property
    def error_file(self) -> Optional[str]:
        return os.path.join(self.local_path, "error.txt") if self.error is not None else None

    def should_stop(self, result: Dict) -> bool:
        return bool(result.get("done"))

    @staticmethod
    def generate_id() -> str:
        import uuid as _uuid

        return _uuid.uuid4().hex[:8]

    def get_json_state(self) -> str:
        return json.dumps({"trial_id": self.trial_id, "config": _jsonable(self.config), "status": self.status,
                           "local_path": self.local_path, "last_result": _jsonable(self.last_result),
                           "checkpoint": self.checkpoint.path if self.checkpoint else None,
                           "resources": self.resources})

    @classmethod
    def from_json_state(cls, json_state: str) -> "Trial":
        d = json.loads(json_state)
        t = cls(d["trial_id"], d["config"], d["local_path"], d.get("resources") or {"CPU": 1})
        t.status, t.last_result = d["status"], d.get("last_result") or {}
        t.checkpoint = _ckpt(d.get("checkpoint"))
        return t


def _flat_cfg(cfg, prefix=""):
    for k, v in (cfg or {}).items():
        if isinstance(v, dict):
            yield from _flat_cfg(v, f"{prefix}{k}/")
        else:
            yield f"{prefix}{k}", v


class ResultGrid:
    def __init__(self, results: List[Result], metric=None, mode=None, experiment_path=None):
        self._results = results
        self._metric = metric
        self._mode = mode
        self.experiment_path = experiment_path

    @property
    def filesystem(self):
        """The filesystem the experiment lives on (local: ``pyarrow.fs.LocalFileSystem`` when
        pyarrow is importable, else None)."""
        try:
            import pyarrow.fs as pafs

            return pafs.LocalFileSystem()
        except Exception:
            return None

    def __len__(self):
        return len(self._results)

    def __getitem__(self, i) -> Result:
        return self._results[i]

    def __iter__(self):
        return iter(self._results)

    @property
    def errors(self):
        return [r.error for r in self._results if r.error is not None]

    @property
    def num_errors(self):
        return len(self.errors)

    @property
    def num_terminated(self):
        return len([r for r in self._results if r.error is None])

    def get_best_result(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last",
                        filter_nan_and_inf: bool = True) -> Result:
        metric = metric or self._metric
        mode = mode or self._mode
        if not metric or not mode:
            raise ValueError("No metric/mode provided to get_best_result and none set in TuneConfig.")
        best, bv = None, None
        for r in self._results:
            if not r.metrics_history and not r.metrics:
                continue
            if scope == "last":
                vals = [r.metrics.get(metric)] if r.metrics else []
            else:
                vals = [m.get(metric) for m in r.metrics_history]
            vals = [v for v in vals if v is not None and (not filter_nan_and_inf or _finite(v))]
            if not vals:
                continue
            v = max(vals) if mode == "max" else min(vals)
            if bv is None or (v > bv if mode == "max" else v < bv):
                best, bv = r, v
        if best is None:
            raise RuntimeError(f"No best trial found for metric {metric}.")
        return best

    def get_dataframe(self, filter_metric=None, filter_mode=None):
        import pandas as pd

        rows = []
        for r in self._results:
            row = dict(r.metrics or {})
            for k, v in (row.pop("config", None) or {}).items():
                row[f"config/{k}"] = v
            row["logdir"] = r.path
            rows.append(row)
        return pd.DataFrame(rows)


def _finite(v):
    try:
        import math

        return math.isfinite(float(v))
    except (TypeError, ValueError):
        return True


class TuneController:
    def __init__(self, trainable, param_space: Dict, tune_config: TuneConfig, run_config: RunConfig,
                 exp_dir: str, restored_trials: Optional[List[Trial]] = None):
        self.trainable = trainable
        self.param_space = param_space or {}
        self.tc = tune_config
        self.rc = run_config
        from .logger import default_logger_callbacks

        # user callbacks + the default CSV / JSON result loggers (progress.csv, params.json)
        self.callbacks = list(run_config.callbacks or []) + default_logger_callbacks(run_config.callbacks)
        self.exp_dir = exp_dir
        os.makedirs(exp_dir, exist_ok=True)
        self.scheduler = tune_config.scheduler or FIFOScheduler()
        self.scheduler.set_search_properties(tune_config.metric, tune_config.mode)
        self.searcher = tune_config.search_alg or BasicVariantGenerator()
        inner = self.searcher
        while isinstance(getattr(inner, "searcher", None), Searcher):  # ConcurrencyLimiter / Repeater
            inner = inner.searcher
        if isinstance(inner, BasicVariantGenerator):
            inner.set_space(self.param_space, tune_config.num_samples)
            self._budget = None  # until exhausted
        else:
            self.searcher.set_search_properties(tune_config.metric, tune_config.mode, self.param_space)
            self._budget = tune_config.num_samples
        self.trials: List[Trial] = list(restored_trials or [])
        self._searcher_done = bool(restored_trials)
        self.kind = self._kind(trainable)
        self.resources = getattr(trainable, "_rca_resources", None) or {"CPU": 1}
        self.max_conc = tune_config.max_concurrent_trials or self._default_concurrency()
        self._t0 = time.time()
        self._stop_all = False
        # TuneConfig.reuse_actors: finished trials' actors, by resource request, for the next trial
        self._actor_cache: Dict[tuple, List] = {}
        self.num_actor_reuses = 0

    # ----------------------------------------------------------------------- helpers
    def _kind(self, t):
        from ..train.data_parallel_trainer import BaseTrainer

        if isinstance(t, BaseTrainer):
            return "trainer"
        if inspect.isclass(t) and issubclass(t, Trainable):
            return "class"
        if callable(t):
            return "function"
        raise TypeError(f"unsupported trainable {t!r}")

    def _default_concurrency(self):
        from .._private.worker import cluster_resources

        if self.kind == "trainer":
            return 1 << 30
        cr = cluster_resources()
        n = 1 << 30
        for k, v in self.resources.items():
            if v > 0:
                n = min(n, int(cr.get(k, 0) // v))
        return max(1, n)

    def get_trial(self, trial_id):
        for t in self.trials:
            if t.trial_id == trial_id:
                return t
        return None

    def _new_trial(self):
        if self._searcher_done:
            return None
        if self._budget is not None and self._budget <= 0:
            self._searcher_done = True
            return None
        tid = uuid.uuid4().hex[:8]
        cfg = self.searcher.suggest(tid)
        if cfg == Searcher.FINISHED:
            self._searcher_done = True
            return None
        if cfg is None:
            return None
        if self._budget is not None:
            self._budget -= 1
        name = f"trial_{len(self.trials):05d}_{tid}"
        if self.tc.trial_dirname_creator:
            name = self.tc.trial_dirname_creator(_TrialView(tid, cfg))
        t = Trial(tid, cfg, os.path.join(self.exp_dir, name), self.resources)
        # TuneConfig.trial_name_creator: the trial's display name (train.get_context().get_trial_name())
        t.trial_name = str(self.tc.trial_name_creator(_TrialView(tid, cfg))) if self.tc.trial_name_creator else name
        os.makedirs(t.local_path, exist_ok=True)
        if getattr(self, "_initial_restore", None):
            t.restore_path = self._initial_restore
        self.trials.append(t)
        self.scheduler.on_trial_add(self, t)
        return t

    def _log_paths(self, trial):
        """RunConfig(log_to_file=True | "file" | ("out", "err")): the trial's stdout / stderr files."""
        ltf = getattr(self.rc, "log_to_file", False)
        if not ltf:
            return None
        names = ("stdout", "stderr") if ltf is True else ((ltf, ltf) if isinstance(ltf, str) else tuple(ltf))
        return os.path.join(trial.local_path, names[0]), os.path.join(trial.local_path, names[1])

    # ----------------------------------------------------------------------- lifecycle
    def _start(self, trial: Trial):
        from .._private.worker import get
        from ..actor import ActorClass
        from ..train._internal.session import TrainContext
        from ..train._internal.worker_group import _TrainWorker

        trial.status = RUNNING
        trial.start_time = time.time()
        os.makedirs(trial.local_path, exist_ok=True)
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_start"):
                cb.on_trial_start(iteration=0, trials=self.trials, trial=trial)
        trial.stop_flag = False
        ckpt = trial.checkpoint if trial.restore_path is None else _ckpt(trial.restore_path)
        trial.restore_path = None
        res = dict(getattr(trial, "resources", None) or self.resources)
        opts = {"num_cpus": res.pop("CPU", 0), "num_gpus": res.pop("GPU", 0), "resources": res or None,
                "max_concurrency": 4}
        opts = {k: v for k, v in opts.items() if v is not None}
        key = self._resource_key(trial)
        if self.kind == "function":
            cached = self._take_cached(key)
            if cached is not None:  # reuse_actors: a finished trial's idle worker actor
                trial.runner = cached
                self.num_actor_reuses += 1
            else:
                trial.runner = ActorClass(_TrainWorker, opts).remote()
            ctx = TrainContext(trial_dir=trial.local_path, trial_id=trial.trial_id,
                               trial_name=getattr(trial, "trial_name", None) or os.path.basename(trial.local_path),
                               experiment_name=os.path.basename(self.exp_dir),
                               metadata={"_ckpt_start": _next_ckpt_index(trial.local_path)})
            fn = self.trainable
            takes = len(inspect.signature(fn).parameters) >= 1
            if not takes:
                fn = (lambda c, f=fn: f())
                takes = True
            logs = self._log_paths(trial)
            if logs:
                fn = _with_log_files(fn, *logs)
            cfg = copy.deepcopy(trial.config)
            # non-blocking: the actor may wait for resources; the first poll queues behind start()
            trial.runner.start.remote(fn, cfg, ctx, ckpt, {})
            trial.pending = trial.runner.poll.remote(0.05)
        elif self.kind == "class":
            cls = ActorClass(_ClassTrainableRunner, {k: v for k, v in opts.items() if k != "max_concurrency"})
            info = {"trial_id": trial.trial_id, "logdir": trial.local_path,
                    "trial_name": getattr(trial, "trial_name", None) or os.path.basename(trial.local_path)}
            cached = self._take_cached(key)
            if cached is not None:
                # reuse_actors: the trainable accepts the new config in place (reset_config -> True)
                try:
                    ok = get(cached.reset.remote(copy.deepcopy(trial.config), ckpt.path if ckpt else None, info,
                                                 self._log_paths(trial)))
                except Exception:  # noqa
                    ok = False
                if ok:
                    trial.runner = cached
                    self.num_actor_reuses += 1
                else:
                    self._kill_quietly(cached)
                    cached = None
            if cached is None:
                trial.runner = cls.remote(self.trainable, copy.deepcopy(trial.config), ckpt.path if ckpt else None,
                                          info, self._log_paths(trial))
            trial.pending = trial.runner.step.remote()
        else:
            trial.thread_q = queue.Queue()
            trainer = self.trainable._with_config(trial.config)
            trainer._in_tune = True
            if ckpt is not None:
                trainer.resume_from_checkpoint = ckpt

            def cb(m, c, trial=trial):
                trial.thread_q.put(("result", m, c))
                return trial.stop_flag

            def run(trial=trial, trainer=trainer):
                try:
                    r = trainer._fit_in_trial(trial.local_path, cb)
                    trial.thread_q.put(("done", r.error))
                except BaseException as e:  # noqa
                    trial.thread_q.put(("done", e))

            th = threading.Thread(target=run, daemon=True)
            th.start()
            trial.runner = th

    def _poll(self, trial: Trial):
        """-> list of events: ("result", metrics, ckpt_path) / ("done", err)."""
        from .._private.worker import get, wait

        if self.kind == "function":
            ready, _ = wait([trial.pending], timeout=0.01)
            if not ready:
                return []
            try:
                r = get(trial.pending)
            except Exception as e:  # noqa - the trial actor died
                return [("done", e)]
            trial.pending = trial.runner.poll.remote(0.05)
            if r[0] == "wait":
                return []
            if r[0] == "result":
                return [("result", r[1], r[2])]
            if r[0] == "done":
                return [("done", None)]
            return [("done", r[1])]
        if self.kind == "class":
            ready, _ = wait([trial.pending], timeout=0.02)
            if not ready:
                return []
            try:
                res = get(trial.pending)
            except Exception as e:  # noqa
                return [("done", e)]
            ck = None
            freq = self.rc.checkpoint_config.checkpoint_frequency
            it = res.get("training_iteration", 0)
            if freq and it % freq == 0:
                ck = get(trial.runner.save.remote(
                    os.path.join(trial.local_path, f"checkpoint_{_next_ckpt_index(trial.local_path):06d}")))
            trial.pending = None
            if res.get("done"):
                return [("result", res, ck), ("done", None)]
            return [("result", res, ck)]
        out = []
        while True:
            try:
                ev = trial.thread_q.get(timeout=0.02 if not out else 0)
            except queue.Empty:
                break
            if ev[0] == "result":
                out.append(("result", ev[1], ev[2].path if ev[2] is not None else None))
            else:
                out.append(("done", ev[1]))
        return out

    # ----------------------------------------------------------------------- actor reuse
    def _resource_key(self, trial: Trial) -> tuple:
        res = dict(getattr(trial, "resources", None) or self.resources)
        return tuple(sorted((k, float(v)) for k, v in res.items()))

    def _take_cached(self, key):
        lst = self._actor_cache.get(key)
        return lst.pop() if lst else None

    @staticmethod
    def _kill_quietly(actor):
        from .._private.worker import kill

        try:
            kill(actor)
        except Exception:
            pass

    def _try_cache(self, trial: Trial) -> bool:
        """``reuse_actors``: keep the actor of a trial that ended cleanly (function trainables:
        only once its training thread has returned) for the next trial with the same resources."""
        from .._private.worker import get

        if not self.tc.reuse_actors or self.kind not in ("function", "class") or trial.runner is None:
            return False
        if sum(len(v) for v in self._actor_cache.values()) >= max(1, self.max_conc):
            return False
        if self.kind == "function":
            try:
                if not get(trial.runner.idle.remote(), timeout=10):
                    return False
            except Exception:  # noqa
                return False
        self._actor_cache.setdefault(self._resource_key(trial), []).append(trial.runner)
        return True

    def _clear_actor_cache(self):
        for lst in self._actor_cache.values():
            for a in lst:
                self._kill_quietly(a)
        self._actor_cache = {}

    def _stop_runner(self, trial: Trial, save=False, reuse=False):
        from .._private.worker import get, kill

        if self.kind in ("function", "class") and trial.runner is not None:
            if save and self.kind == "class":
                try:
                    p = get(trial.runner.save.remote(os.path.join(
                        trial.local_path, f"checkpoint_{_next_ckpt_index(trial.local_path):06d}")))
                    self._register_ckpt(trial, p, trial.last_result)
                except Exception:
                    pass
            if reuse and self._try_cache(trial):
                trial.runner = None
                return
            try:
                kill(trial.runner)
            except Exception:
                pass
        elif self.kind == "trainer" and trial.runner is not None:
            trial.stop_flag = True
            trial.runner.join(timeout=60)
        trial.runner = None

    def exploit(self, trial: Trial, donor: Trial, new_config: Dict):
        """PBT: restart ``trial`` from ``donor``'s latest checkpoint with ``new_config``."""
        self._stop_runner(trial)
        dst = os.path.join(trial.local_path, f"checkpoint_{_next_ckpt_index(trial.local_path):06d}")
        shutil.copytree(donor.checkpoint.path, dst, dirs_exist_ok=True)
        trial.config = new_config
        trial.restore_path = dst
        trial.checkpoint = _ckpt(dst)
        trial.iteration_offset = trial.last_result.get("training_iteration", 0)
        trial.status = PENDING

    # ------------------------------------------------------------ scheduler hooks
    def unpause(self, trial: Trial):
        """A PAUSED trial goes back to PENDING and resumes from its last checkpoint."""
        if trial.status != PAUSED:
            return
        trial.status = PENDING
        if hasattr(self.searcher, "on_unpause"):
            self.searcher.on_unpause(trial.trial_id)
        trial.restore_path = trial.checkpoint.path if trial.checkpoint else None
        trial.iteration_offset = trial.last_result.get("training_iteration", 0) if trial.checkpoint else 0

    def stop_paused(self, trial: Trial):
        """Terminate a PAUSED trial (e.g. cut by synchronous successive halving)."""
        if trial.status == PAUSED:
            self._complete(trial)

    def restart(self, trial: Trial, new_config: Optional[Dict] = None, new_resources: Optional[Dict] = None):
        """Checkpoint a RUNNING trial, stop it and queue it again with a new config and/or
        resources (ResourceChangingScheduler, PopulationBasedTrainingReplay); it resumes from that
        checkpoint in a fresh trial actor sized by ``new_resources``."""
        self._stop_runner(trial, save=True)
        if new_config is not None:
            trial.config = new_config
        if new_resources is not None:
            trial.resources = dict(new_resources)
        trial.status = PENDING
        trial.restore_path = trial.checkpoint.path if trial.checkpoint else None
        trial.iteration_offset = trial.last_result.get("training_iteration", 0) if trial.checkpoint else 0

    @property
    def searcher_done(self) -> bool:
        return bool(self._searcher_done)

    def _should_stop(self, trial, result) -> bool:
        stop_trial, stop_all = evaluate_stop(self.rc.stop, trial.trial_id, result)
        if stop_all:
            self._stop_all = True
        return stop_trial

    def _on_result(self, trial: Trial, metrics: Dict, ckpt_path: Optional[str]):
        m = dict(metrics)
        _add_flat_keys(m)
        if trial.iteration_offset:
            m["training_iteration"] = m.get("training_iteration", 0) + trial.iteration_offset
        m.setdefault("training_iteration", len(trial.metrics_history) + 1)
        m["trial_id"] = trial.trial_id
        m["time_total_s"] = time.time() - trial.start_time
        m["timestamp"] = time.time()
        m["config"] = trial.config
        trial.last_result = m
        trial.metrics_history.append(m)
        if ckpt_path:
            self._register_ckpt(trial, ckpt_path, m)
        with open(os.path.join(trial.local_path, "result.json"), "a") as f:
            f.write(json.dumps(_jsonable(m)) + "\n")
        self.searcher.on_trial_result(trial.trial_id, m)
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_result"):
                cb.on_trial_result(iteration=0, trials=self.trials, trial=trial, result=m)
        if self._should_stop(trial, m):
            return TrialScheduler.STOP
        return self.scheduler.on_trial_result(self, trial, m)

    def _register_ckpt(self, trial: Trial, path: str, metrics: Dict):
        """A new persisted checkpoint of ``trial``: it becomes the trial's latest, and
        CheckpointConfig(num_to_keep, checkpoint_score_attribute) prunes the older ones (the
        latest always stays, for resume) -- reference: tune/execution/tune_controller.py +
        train/_internal/checkpoint_manager.py."""
        from ..train._internal.backend_executor import CheckpointManager

        trial.checkpoint = _ckpt(path)
        mgr = getattr(trial, "_ckpt_mgr", None)
        if mgr is None:
            mgr = trial._ckpt_mgr = CheckpointManager(self.rc.checkpoint_config)
        mgr.register(trial.checkpoint, dict(metrics or {}))

    def _save_at_end(self, trial: Trial) -> bool:
        """CheckpointConfig(checkpoint_at_end=True): a class trainable that ends cleanly saves
        once more unless its last result was just checkpointed."""
        if self.kind != "class" or not self.rc.checkpoint_config.checkpoint_at_end:
            return False
        mgr = getattr(trial, "_ckpt_mgr", None)
        return not (mgr and mgr.entries and mgr.entries[-1][1].get("training_iteration")
                    == trial.last_result.get("training_iteration"))

    def _complete(self, trial: Trial, err=None):
        if err is not None:
            trial.num_failures += 1
            mf = self.rc.failure_config.max_failures
            if mf < 0 or trial.num_failures <= mf:
                trial.status = PENDING
                trial.restore_path = trial.checkpoint.path if trial.checkpoint else None
                trial.iteration_offset = trial.last_result.get("training_iteration", 0) if trial.checkpoint else 0
                return
            trial.status = ERROR
            trial.error = err
            self.scheduler.on_trial_error(self, trial)
            self.searcher.on_trial_complete(trial.trial_id, trial.last_result, error=True)
            if self.rc.failure_config.fail_fast:
                self._stop_all = True
        else:
            trial.status = TERMINATED
            self.scheduler.on_trial_complete(self, trial, trial.last_result)
            self.searcher.on_trial_complete(trial.trial_id, trial.last_result)
        for cb in self.callbacks:
            if hasattr(cb, "on_trial_complete"):
                cb.on_trial_complete(iteration=0, trials=self.trials, trial=trial)

    def run(self):
        from .._private import worker as w

        if not w.is_initialized():
            w.init()
        while True:
            if self.tc.time_budget_s and time.time() - self._t0 > self.tc.time_budget_s:
                self._stop_all = True
            running = [t for t in self.trials if t.status == RUNNING]
            if self._stop_all:
                for t in running:
                    self._stop_runner(t)
                    t.status = TERMINATED
                break
            # launch
            while len(running) < self.max_conc:
                t = next((x for x in self.trials if x.status == PENDING), None)
                if t is None:
                    t = self._new_trial()
                if t is None:
                    break
                self._start(t)
                running.append(t)
            if not running:
                # everything left may be PAUSED: let the scheduler (or the generic rule) resume some
                if self._resume_paused() and any(x.status == PENDING for x in self.trials):
                    continue
                if self._searcher_done or all(t.status in (TERMINATED, ERROR) for t in self.trials) and \
                        self._new_trial_blocked():
                    break
                time.sleep(0.01)
                continue
            for t in running:
                if t.status != RUNNING:
                    continue
                for ev in self._poll(t):
                    if ev[0] == "result":
                        decision = self._on_result(t, ev[1], ev[2])
                        if decision == TrialScheduler.STOP:
                            self._stop_runner(t, save=self._save_at_end(t), reuse=True)
                            self._complete(t)
                            break
                        if decision == TrialScheduler.PAUSE:
                            self._stop_runner(t, save=True, reuse=True)
                            t.status = PAUSED
                            if hasattr(self.searcher, "on_pause"):  # frees a ConcurrencyLimiter slot
                                self.searcher.on_pause(t.trial_id)
                            break
                        if decision == TrialScheduler.NOOP:
                            break  # exploit() already restarted the trial
                        if self.kind == "class" and t.status == RUNNING and t.runner is not None:
                            t.pending = t.runner.step.remote()
                    else:
                        self._stop_runner(t, save=ev[1] is None and self._save_at_end(t), reuse=ev[1] is None)
                        self._complete(t, ev[1])
                        break
            self._save_state()
            self._resume_paused()
        self._clear_actor_cache()
        self._save_state()
        return self._results()

    def _resume_paused(self) -> bool:
        """Schedulers that pace trials themselves (synchronous HyperBand) get a hook every pass;
        for the others, PAUSED trials resume when nothing else is pending. True if any trial
        is PAUSED."""
        self.scheduler.choose_trial_to_run(self)
        if (not getattr(self.scheduler, "manages_paused_trials", False)
                and not any(x.status in (PENDING,) for x in self.trials) and self._searcher_done):
            for x in self.trials:
                if x.status == PAUSED and len([y for y in self.trials if y.status == RUNNING]) < self.max_conc:
                    x.status = PENDING
                    if hasattr(self.searcher, "on_unpause"):
                        self.searcher.on_unpause(x.trial_id)
                    x.restore_path = x.checkpoint.path if x.checkpoint else None
                    x.iteration_offset = x.last_result.get("training_iteration", 0)
        return any(x.status in (PAUSED, PENDING) for x in self.trials)

    def _new_trial_blocked(self):
        return self._searcher_done

    def _results(self):
        out = []
        for t in self.trials:
            mgr = getattr(t, "_ckpt_mgr", None)
            out.append(Result(metrics=t.last_result or None, checkpoint=t.checkpoint, error=t.error,
                              path=t.local_path, metrics_history=t.metrics_history,
                              best_checkpoints=list(mgr.entries) if mgr else []))
        return ResultGrid(out, self.tc.metric, self.tc.mode, self.exp_dir)

    def _save_state(self):
        st = {"trials": [{"trial_id": t.trial_id, "config": _jsonable(t.config), "status": t.status,
                          "local_path": t.local_path, "last_result": _jsonable(t.last_result),
                          "checkpoint": t.checkpoint.path if t.checkpoint else None,
                          "error": repr(t.error) if t.error else None} for t in self.trials]}
        tmp = os.path.join(self.exp_dir, ".experiment_state.json.tmp")
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, os.path.join(self.exp_dir, "experiment_state.json"))


class _TrialView:
    def __init__(self, tid, cfg):
        self.trial_id = tid
        self.config = cfg


def _ckpt(path):
    from ..train._checkpoint import Checkpoint

    return Checkpoint.from_directory(path) if path else None


def _next_ckpt_index(path):
    if not os.path.isdir(path):
        return 0
    idx = [int(d.split("_")[-1]) for d in os.listdir(path) if d.startswith("checkpoint_") and d.split("_")[-1].isdigit()]
    return max(idx) + 1 if idx else 0


def _jsonable(d):
    out = {}
    for k, v in (d or {}).items():
        try:
            json.dumps(v)
            out[k] = v
        except TypeError:
            out[k] = _jsonable(v) if isinstance(v, dict) else repr(v)
    return out


class Tuner:
    def __init__(self, trainable=None, *, param_space: Optional[Dict] = None, tune_config: Optional[TuneConfig] = None,
                 run_config: Optional[RunConfig] = None, _restored_trials=None, _exp_dir=None):
        from .registry import resolve_trainable

        self.trainable = resolve_trainable(trainable)  # a name from tune.register_trainable works too
        if param_space is not None and not isinstance(param_space, dict) and hasattr(param_space, "to_dict"):
            param_space = param_space.to_dict()  # an RLlib AlgorithmConfig (its search-space leaves kept)
        self.param_space = param_space or {}
        self.tune_config = tune_config or TuneConfig()
        from ..train.data_parallel_trainer import BaseTrainer

        if run_config is None and isinstance(trainable, BaseTrainer):
            run_config = trainable.run_config
        self.run_config = run_config or RunConfig()
        self._restored = _restored_trials
        self._exp_dir = _exp_dir

    def fit(self) -> ResultGrid:
        name = self.run_config.name or f"{_tname(self.trainable)}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        exp_dir = self._exp_dir or os.path.join(os.path.expanduser(self.run_config.storage_path), name)
        rc = self.run_config
        rep = getattr(rc, "progress_reporter", None)
        if rep is not None and rep not in (rc.callbacks or []):
            rc.callbacks = list(rc.callbacks or []) + [rep]
        ctrl = TuneController(self.trainable, self.param_space, self.tune_config, rc, exp_dir, self._restored)
        ctrl._initial_restore = getattr(self, "_initial_restore", None)  # tune.run(restore=<checkpoint dir>)
        grid = ctrl.run()
        for cb in (rc.callbacks or []):
            if hasattr(cb, "on_experiment_end"):
                cb.on_experiment_end(trials=ctrl.trials)
        return grid

    def get_results(self) -> ResultGrid:
        return self.fit()

    @classmethod
    def can_restore(cls, path: str) -> bool:
        return os.path.exists(os.path.join(path, "experiment_state.json"))

    @classmethod
    def restore(cls, path: str, trainable, *, param_space=None, resume_unfinished=True, resume_errored=False,
                restart_errored=False, tune_config=None, run_config=None) -> "Tuner":
        with open(os.path.join(path, "experiment_state.json")) as f:
            st = json.load(f)
        trials = []
        for d in st["trials"]:
            t = Trial(d["trial_id"], d["config"], d["local_path"], {"CPU": 1})
            t.last_result = d["last_result"] or {}
            t.checkpoint = _ckpt(d["checkpoint"])
            hp = os.path.join(t.local_path, "result.json")
            if os.path.exists(hp):
                with open(hp) as f:
                    t.metrics_history = [json.loads(l) for l in f if l.strip()]
            status = d["status"]
            if status == TERMINATED:
                t.status = TERMINATED
            elif status == ERROR and not (resume_errored or restart_errored):
                t.status = ERROR
                t.error = RuntimeError(d.get("error") or "trial errored")
            elif status != ERROR and not resume_unfinished:  # ResumeConfig(unfinished=SKIP)
                t.status = TERMINATED
            else:
                t.status = PENDING
                if not restart_errored and t.checkpoint is not None:
                    t.restore_path = t.checkpoint.path
                    t.iteration_offset = t.last_result.get("training_iteration", 0)
            trials.append(t)
        return cls(trainable, param_space=param_space, tune_config=tune_config, run_config=run_config,
                   _restored_trials=trials, _exp_dir=path)


def _redirect_fds(out_path, err_path):
    """Point this process's file descriptors 1 and 2 at the trial's log files (appending), so
    output from C extensions and child processes lands there too, not only Python-level writes.
    Returns the saved descriptors for ``_restore_fds``."""
    import sys

    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    sys.stdout.flush()
    sys.stderr.flush()
    saved = (os.dup(1), os.dup(2))
    fo = os.open(out_path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
    fe = fo if err_path == out_path else os.open(err_path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
    os.dup2(fo, 1)
    os.dup2(fe, 2)
    os.close(fo)
    if fe != fo:
        os.close(fe)
    return saved


def _restore_fds(saved):
    import sys

    sys.stdout.flush()
    sys.stderr.flush()
    os.dup2(saved[0], 1)
    os.dup2(saved[1], 2)
    os.close(saved[0])
    os.close(saved[1])


def _with_log_files(fn, out_path, err_path):
    """Run ``fn(config)`` with this process's stdout / stderr (descriptors 1 and 2) appended to
    the trial's log files; the worker's own descriptors come back afterwards."""

    def run(config):
        saved = _redirect_fds(out_path, err_path)
        try:
            return fn(config)
        finally:
            _restore_fds(saved)

    run.__name__ = getattr(fn, "__name__", "trainable")
    return run


def _tname(t):
    return getattr(t, "__name__", type(t).__name__)
