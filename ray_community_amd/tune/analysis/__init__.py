"""ExperimentAnalysis: what ``tune.run`` returns (reference:
python/ray/tune/analysis/experiment_analysis.py:46).

Built over a finished experiment's ResultGrid, or loaded from an experiment directory on disk
(``ExperimentAnalysis(path)`` reads ``experiment_state.json`` and each trial's ``result.json``).
Trials are exposed as light records with the attributes the legacy API hands out
(``trial_id``, ``config``, ``last_result``, ``path`` / ``local_path`` / ``logdir``, ``checkpoint``,
``status``, ``error``), so ``analysis.trials[i].last_result[...]`` code keeps working."""
from __future__ import annotations

import json
import math
import os
from typing import Any, Dict, List, Optional, Union


def _finite(v) -> bool:
    try:
        return math.isfinite(float(v))
    except (TypeError, ValueError):
        return False


class AnalysisTrial:
    """One trial of a finished experiment (the subset of ``tune.experiment.Trial`` analysis needs)."""

    def __init__(self, trial_id: str, config: Dict, last_result: Dict, path: str, checkpoint=None,
                 error=None, metrics_history: Optional[List[Dict]] = None, checkpoints=None):
        self.trial_id = trial_id
        self.config = config or {}
        self.last_result = last_result or {}
        self.path = self.local_path = self.logdir = path
        self.checkpoint = checkpoint
        self.error = error
        self.status = "ERROR" if error is not None else "TERMINATED"
        self.metrics_history = list(metrics_history or [])
        self._checkpoints = list(checkpoints or [])  # [(Checkpoint, metrics)]

    @property
    def metrics(self) -> Dict:  # the Result-style name of last_result
        return self.last_result

    def __repr__(self):
        return f"Trial({self.trial_id}, {self.status})"

    def __str__(self):
        return self.trial_id


class ExperimentAnalysis:
    def __init__(self, experiment_checkpoint_path: Union[str, Any], trials: Optional[List[AnalysisTrial]] = None,
                 default_metric: Optional[str] = None, default_mode: Optional[str] = None, *, metric=None,
                 mode=None):
        from ..tuner import ResultGrid

        self.default_metric = default_metric or metric
        self.default_mode = default_mode or mode
        if self.default_mode not in (None, "min", "max"):
            raise ValueError("`mode` must be one of ['min', 'max']")
        if isinstance(experiment_checkpoint_path, ResultGrid):
            grid = experiment_checkpoint_path
            self._experiment_path = grid.experiment_path
            self._trials = trials or [self._from_result(r) for r in grid]
        else:
            self._experiment_path = os.path.expanduser(str(experiment_checkpoint_path))
            self._trials = trials or self._load_trials(self._experiment_path)

    # ----------------------------------------------------------------------- loading
    @staticmethod
    def _from_result(r) -> AnalysisTrial:
        m = dict(r.metrics or {})
        return AnalysisTrial(m.get("trial_id") or os.path.basename(r.path or ""), r.config, m, r.path,
                             r.checkpoint, r.error, r.metrics_history, getattr(r, "best_checkpoints", None))

    @staticmethod
    def _load_trials(path: str) -> List[AnalysisTrial]:
        from ...train._checkpoint import Checkpoint

        state = os.path.join(path, "experiment_state.json")
        if not os.path.exists(state):
            raise ValueError(f"No experiment state found under {path!r}")
        with open(state) as f:
            st = json.load(f)
        out = []
        for d in st["trials"]:
            hist = []
            rp = os.path.join(d["local_path"], "result.json")
            if os.path.exists(rp):
                with open(rp) as f:
                    hist = [json.loads(l) for l in f if l.strip()]
            ck = Checkpoint.from_directory(d["checkpoint"]) if d.get("checkpoint") else None
            err = RuntimeError(d["error"]) if d.get("error") else None
            out.append(AnalysisTrial(d["trial_id"], d["config"], d.get("last_result") or (hist[-1] if hist else {}),
                                     d["local_path"], ck, err, hist))
        return out

    # ----------------------------------------------------------------------- helpers
    def _metric(self, metric):
        metric = metric or self.default_metric
        if not metric:
            raise ValueError("No `metric` given and no default metric set (pass metric= to tune.run)")
        return metric

    def _mode(self, mode):
        mode = mode or self.default_mode
        if mode not in ("min", "max"):
            raise ValueError("No `mode` given and no default mode set (pass mode='min'|'max' to tune.run)")
        return mode

    @staticmethod
    def _score(trial: AnalysisTrial, metric: str, mode: str, scope: str, filter_nan_and_inf: bool):
        if scope == "last":
            vals = [trial.last_result.get(metric)]
        elif scope in ("all", "last-5-avg", "last-10-avg", "avg"):
            vals = [m.get(metric) for m in trial.metrics_history] or [trial.last_result.get(metric)]
        else:
            raise ValueError(f"scope must be one of last, avg, last-5-avg, last-10-avg, all; got {scope!r}")
        vals = [v for v in vals if v is not None and (not filter_nan_and_inf or _finite(v))]
        if not vals:
            return None
        if scope == "avg":
            return sum(vals) / len(vals)
        if scope in ("last-5-avg", "last-10-avg"):
            n = 5 if scope == "last-5-avg" else 10
            return sum(vals[-n:]) / len(vals[-n:])
        if scope == "all":
            return max(vals) if mode == "max" else min(vals)
        return vals[-1]

    # ----------------------------------------------------------------------- API
    @property
    def trials(self) -> List[AnalysisTrial]:
        return list(self._trials)

    @property
    def experiment_path(self) -> Optional[str]:
        return self._experiment_path

    def get_best_trial(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last",
                       filter_nan_and_inf: bool = True) -> Optional[AnalysisTrial]:
        metric, mode = self._metric(metric), self._mode(mode)
        best, bv = None, None
        for t in self._trials:
            v = self._score(t, metric, mode, scope, filter_nan_and_inf)
            if v is None:
                continue
            if bv is None or (v > bv if mode == "max" else v < bv):
                best, bv = t, v
        return best

    def get_best_config(self, metric: Optional[str] = None, mode: Optional[str] = None,
                        scope: str = "last") -> Optional[Dict]:
        t = self.get_best_trial(metric, mode, scope)
        return t.config if t else None

    def get_last_checkpoint(self, trial: Optional[AnalysisTrial] = None, metric: str = "training_iteration",
                            mode: str = "max"):
        trial = trial or self.best_trial
        if trial is None:
            return None
        if trial._checkpoints:
            return self.get_best_checkpoint(trial, metric, mode)
        return trial.checkpoint

    def _get_trial_checkpoints_with_metric(self, trial: AnalysisTrial, metric: Optional[str] = None):
        metric = metric or self.default_metric or "training_iteration"
        if trial._checkpoints:
            return [(c, m.get(metric)) for c, m in trial._checkpoints]
        return [(trial.checkpoint, trial.last_result.get(metric))] if trial.checkpoint else []

    def get_best_checkpoint(self, trial: AnalysisTrial, metric: Optional[str] = None, mode: Optional[str] = None):
        metric, mode = self._metric(metric), self._mode(mode)
        scored = [(v, c) for c, v in self._get_trial_checkpoints_with_metric(trial, metric)
                  if v is not None and _finite(v)]
        if not scored:
            return None
        return (max if mode == "max" else min)(scored, key=lambda x: x[0])[1]

    def get_all_configs(self, prefix: bool = False) -> Dict[str, Dict]:
        if prefix:
            return {t.path: {f"config/{k}": v for k, v in t.config.items()} for t in self._trials}
        return {t.path: t.config for t in self._trials}

    @property
    def best_trial(self) -> Optional[AnalysisTrial]:
        return self.get_best_trial()

    @property
    def best_config(self) -> Optional[Dict]:
        return self.get_best_config()

    @property
    def best_checkpoint(self):
        t = self.best_trial
        if t is None:
            return None
        return self.get_best_checkpoint(t) if t._checkpoints else t.checkpoint

    @property
    def best_result(self) -> Optional[Dict]:
        t = self.best_trial
        return t.last_result if t else None

    @property
    def best_path(self) -> Optional[str]:
        t = self.best_trial
        return t.path if t else None

    best_logdir = best_path

    @property
    def best_dataframe(self):
        return self.trial_dataframes[self.best_path]

    @property
    def best_result_df(self):
        import pandas as pd

        return pd.DataFrame([self.best_result])

    @property
    def results(self) -> Dict[str, Dict]:
        return {t.trial_id: t.last_result for t in self._trials}

    def _row(self, result: Dict, trial: AnalysisTrial) -> Dict:
        row = {k: v for k, v in result.items() if k != "config"}
        for k, v in trial.config.items():
            row[f"config/{k}"] = v
        row["logdir"] = trial.path
        return row

    @property
    def results_df(self):
        import pandas as pd

        return pd.DataFrame([self._row(t.last_result, t) for t in self._trials])

    @property
    def trial_dataframes(self) -> Dict[str, Any]:
        import pandas as pd

        return {t.path: pd.DataFrame([{k: v for k, v in m.items() if k != "config"} for m in t.metrics_history])
                for t in self._trials}

    def dataframe(self, metric: Optional[str] = None, mode: Optional[str] = None):
        """One row per trial: its last result, or (metric and mode given) its best result."""
        import pandas as pd

        rows = []
        for t in self._trials:
            res = t.last_result
            if metric and mode and t.metrics_history:
                cands = [m for m in t.metrics_history if _finite(m.get(metric))]
                if cands:
                    res = (max if mode == "max" else min)(cands, key=lambda m: float(m[metric]))
            rows.append(self._row(res, t))
        return pd.DataFrame(rows)

    def stats(self) -> Dict:
        return {"num_trials": len(self._trials), "num_errors": sum(t.error is not None for t in self._trials)}


__all__ = ["ExperimentAnalysis", "AnalysisTrial"]
