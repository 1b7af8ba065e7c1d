"""Data-parallel GBDT trainers, checkpoints, report callbacks and predictors.

Reference parity:
``python/ray/train/xgboost/xgboost_trainer.py:18-67`` (per-worker function: resume from the
checkpoint's model for the REMAINING rounds, train shard -> DMatrix, every non-train dataset is an
eval set, train metrics included), ``:70-190`` (constructor: ``label_column``, ``params``,
``num_boost_round`` = target total rounds, default report callback honouring
``CheckpointConfig.checkpoint_frequency`` / ``checkpoint_at_end``, ``get_model``, a ``"train"``
dataset is required), ``python/ray/train/xgboost/_xgboost_utils.py`` (``RayTrainReportCallback``:
``{eval_name}-{metric}`` keys of the latest round, optional metric selection / renaming, checkpoint
every ``frequency`` rounds and at the end), ``xgboost_checkpoint.py`` / ``xgboost_predictor.py``
and the lightgbm counterparts.

The workers form a torch.distributed group (RCCL on GPU, gloo on CPU) through the TorchConfig
backend; the boosting itself is ``train/gbdt/core.py`` with histograms from the gfx950 kernel when
the workers hold GPUs.
"""
from __future__ import annotations

import os
import tempfile
from functools import partial
from typing import Any, Dict, List, Optional, Union

import numpy as np

from .._checkpoint import Checkpoint
from ..data_parallel_trainer import DataParallelTrainer
from ..torch.config import TorchConfig
from .core import Booster, DMatrix, TrainingCallback, train

TRAIN_DATASET_KEY = "train"


class GBDTCheckpoint(Checkpoint):
    """Directory checkpoint holding a boosted model as JSON (``model.json``)."""

    MODEL_FILENAME = "model.json"

    @classmethod
    def from_model(cls, booster: Booster, *, preprocessor=None, path: Optional[str] = None):
        path = path or tempfile.mkdtemp(prefix="rca_gbdt_ckpt_")
        os.makedirs(path, exist_ok=True)
        booster.save_model(os.path.join(path, cls.MODEL_FILENAME))
        ck = cls(path)
        if preprocessor is not None:
            import cloudpickle

            with open(os.path.join(path, "preprocessor.pkl"), "wb") as f:
                cloudpickle.dump(preprocessor, f)
        return ck

    def get_model(self) -> Booster:
        return Booster().load_model(os.path.join(self.path, self.MODEL_FILENAME))

    def get_preprocessor(self):
        p = os.path.join(self.path, "preprocessor.pkl")
        if not os.path.exists(p):
            return None
        import cloudpickle

        with open(p, "rb") as f:  # written by from_model above
            return cloudpickle.load(f)


class RayTrainReportCallback(TrainingCallback):
    """Reports the latest round's eval metrics (``{eval_name}-{metric}``) through ``train.report``
    on every worker, with a checkpoint from rank 0 every ``frequency`` rounds and at the end."""

    CHECKPOINT_NAME = GBDTCheckpoint.MODEL_FILENAME

    def __init__(self, metrics: Optional[Union[str, List[str], Dict[str, str]]] = None,
                 filename: str = GBDTCheckpoint.MODEL_FILENAME, frequency: int = 0, checkpoint_at_end: bool = True,
                 results_postprocessing_fn=None):
        self._metrics = [metrics] if isinstance(metrics, str) else metrics
        self._filename = filename
        self._frequency = int(frequency or 0)
        self._checkpoint_at_end = checkpoint_at_end
        self._post = results_postprocessing_fn
        self._last_report: Optional[Dict[str, Any]] = None
        self._last_ckpt_iter = -1
        self._iter = -1

    @classmethod
    def get_model(cls, checkpoint: Checkpoint, filename: str = GBDTCheckpoint.MODEL_FILENAME) -> Booster:
        return Booster().load_model(os.path.join(checkpoint.path, filename))

    def _flat(self, evals_log) -> Dict[str, Any]:
        flat = {f"{name}-{met}": vals[-1] for name, d in evals_log.items() for met, vals in d.items()}
        if self._metrics is None:
            out = flat
        elif isinstance(self._metrics, dict):
            out = {k: flat[v] for k, v in self._metrics.items() if v in flat}
        else:
            out = {k: flat[k] for k in self._metrics if k in flat}
        return self._post(out) if self._post else out

    def _checkpoint(self, model: Booster):
        from .. import get_context

        if get_context().get_world_rank() != 0:
            return None
        d = tempfile.mkdtemp(prefix="rca_gbdt_report_")
        model.save_model(os.path.join(d, self._filename))
        return GBDTCheckpoint(d)

    def after_iteration(self, model, epoch, evals_log) -> bool:
        from .. import report

        self._iter = epoch
        self._last_report = self._flat(evals_log)
        ck = None
        if self._frequency > 0 and (epoch + 1) % self._frequency == 0:
            ck = self._checkpoint(model)
            self._last_ckpt_iter = epoch
        report(dict(self._last_report), checkpoint=ck)
        return False

    def after_training(self, model):
        from .. import report

        if self._checkpoint_at_end and self._iter >= 0 and self._last_ckpt_iter != self._iter:
            report(dict(self._last_report or {}), checkpoint=self._checkpoint(model))
        return model


def _frame_xy(df, label_column: str):
    return df.drop(columns=[label_column]), df[label_column]


def _gbdt_train_fn_per_worker(config: dict, label_column: str, num_boost_round: int, dataset_keys: set,
                              train_kwargs: dict, flavor: str, use_gpu: bool):
    import torch

    from .. import get_checkpoint, get_dataset_shard

    dev = "cpu"
    if use_gpu and torch.cuda.is_available():
        dev = f"cuda:{torch.cuda.current_device()}"
    ck = get_checkpoint()
    start_model, remaining = None, num_boost_round
    if ck is not None:
        start_model = RayTrainReportCallback.get_model(ck)
        remaining = num_boost_round - start_model.num_boosted_rounds()
    train_df = get_dataset_shard(TRAIN_DATASET_KEY).materialize().to_pandas()
    X, y = _frame_xy(train_df, label_column)
    dtrain = DMatrix(X, label=y, device=dev)
    evals = [(dtrain, TRAIN_DATASET_KEY)]
    for k in sorted(dataset_keys - {TRAIN_DATASET_KEY}):
        df = get_dataset_shard(k).materialize().to_pandas()
        ex, ey = _frame_xy(df, label_column)
        evals.append((DMatrix(ex, label=ey, device=dev), k))
    kw = dict(train_kwargs)
    cbs = list(kw.pop("callbacks", []))
    train(config, dtrain, num_boost_round=max(0, remaining), evals=evals, xgb_model=start_model, callbacks=cbs,
          flavor=flavor, **kw)


class GBDTConfig(TorchConfig):
    """Backend of the GBDT trainers: the workers' collective group for histogram all-reduces
    (RCCL on GPU workers, gloo on CPU). Stands in for the reference's ``XGBoostConfig``
    (``xgboost_communicator="rabit"``) / lightgbm network setup; ``"rabit"`` is accepted as an
    alias of the default."""

    def __init__(self, xgboost_communicator: str = "rabit", backend=None, timeout_s: int = 1800):
        if xgboost_communicator not in ("rabit", "rccl", "nccl", "gloo"):
            raise NotImplementedError(f"Unsupported backend: {xgboost_communicator}")
        super().__init__()
        self.xgboost_communicator = xgboost_communicator
        self.backend = backend or ({"rccl": "nccl", "nccl": "nccl", "gloo": "gloo"}.get(xgboost_communicator))
        self.timeout_s = timeout_s


class _GBDTTrainer(DataParallelTrainer):
    _flavor = "xgboost"

    def __init__(self, train_loop_per_worker=None, *, datasets: Optional[Dict[str, Any]] = None,
                 label_column: Optional[str] = None, params: Optional[Dict[str, Any]] = None,
                 num_boost_round: int = 10, scaling_config=None, run_config=None, dataset_config=None,
                 resume_from_checkpoint=None, metadata=None, train_loop_config=None, xgboost_config=None,
                 lightgbm_config=None, **train_kwargs):
        from ...air.config import RunConfig, ScalingConfig

        if train_loop_per_worker is not None:
            # the reference's v2 form: the user's loop calls ``train(...)`` with a report callback
            self._v2 = True
            self.label_column, self.params, self.num_boost_round = label_column, dict(params or {}), num_boost_round
            DataParallelTrainer.__init__(self, train_loop_per_worker, train_loop_config=train_loop_config,
                                         backend_config=xgboost_config or lightgbm_config or GBDTConfig(),
                                         scaling_config=scaling_config, run_config=run_config, datasets=datasets,
                                         dataset_config=dataset_config, resume_from_checkpoint=resume_from_checkpoint,
                                         metadata=metadata)
            return
        self._v2 = False
        if label_column is None:
            raise TypeError("label_column is required (or pass a train_loop_per_worker)")
        if TRAIN_DATASET_KEY not in (datasets or {}):
            raise KeyError(f"'{TRAIN_DATASET_KEY}' key must be preset in `datasets`. Got {list((datasets or {}))}")
        run_config = run_config or RunConfig()
        scaling_config = scaling_config or ScalingConfig()
        cbs = list(train_kwargs.get("callbacks", []) or [])
        if not any(isinstance(c, RayTrainReportCallback) for c in cbs):
            cc = getattr(run_config, "checkpoint_config", None)
            freq = getattr(cc, "checkpoint_frequency", 0) if cc is not None else 0
            at_end = getattr(cc, "checkpoint_at_end", None) if cc is not None else None
            cbs.append(self._report_callback_cls()(frequency=freq or 0,
                                                  checkpoint_at_end=True if at_end is None else at_end))
        train_kwargs["callbacks"] = cbs
        self.label_column = label_column
        self.params = dict(params or {})
        self.num_boost_round = num_boost_round
        self._fn_args = dict(label_column=label_column, num_boost_round=num_boost_round,
                             dataset_keys=set(datasets), train_kwargs=train_kwargs, flavor=self._flavor,
                             use_gpu=bool(getattr(scaling_config, "use_gpu", False)))
        fn = partial(_gbdt_train_fn_per_worker, **self._fn_args)
        super().__init__(_as_one_arg(fn), train_loop_config=self.params, backend_config=TorchConfig(),
                         scaling_config=scaling_config, run_config=run_config, datasets=datasets,
                         dataset_config=dataset_config, resume_from_checkpoint=resume_from_checkpoint,
                         metadata=metadata)

    @classmethod
    def _report_callback_cls(cls):
        return RayTrainReportCallback

    @classmethod
    def get_model(cls, checkpoint: Checkpoint) -> Booster:
        return RayTrainReportCallback.get_model(checkpoint)

    def _with_config(self, config):
        if getattr(self, "_v2", False):
            return DataParallelTrainer._with_config(self, config)
        return self._with_params(config)

    def _with_params(self, config):
        """A Tune trial's config: ``{"params": {...}}`` overrides booster parameters (the reference's
        ``Tuner(XGBoostTrainer(...), param_space={"params": {...}})``), ``num_boost_round`` too."""
        import copy

        t = copy.copy(self)
        cfg = dict(self.train_loop_config or {})
        if isinstance(config, dict):
            cfg.update(config.get("params", {}) or {})
            cfg.update(config.get("train_loop_config", {}) or {})
        t.train_loop_config = cfg
        t.params = cfg
        if isinstance(config, dict) and "num_boost_round" in config:
            t.num_boost_round = int(config["num_boost_round"])
            fn = self._fn_args
            t.train_loop_per_worker = _as_one_arg(partial(_gbdt_train_fn_per_worker, **dict(
                fn, num_boost_round=t.num_boost_round)))
        return t


def _as_one_arg(fn):
    def train_loop_per_worker(config):
        return fn(config)

    return train_loop_per_worker


class GBDTPredictor:
    """Batch inference with a boosted model (numpy / pandas / dict batches, ``map_batches``
    friendly); ``{"predictions": ...}`` like the reference's predictors."""

    def __init__(self, model: Booster, preprocessor=None, use_gpu: bool = False):
        self.model = model
        self.preprocessor = preprocessor
        self.device = "cpu"
        if use_gpu:
            import torch

            if torch.cuda.is_available():
                self.device = "cuda"

    @classmethod
    def from_checkpoint(cls, checkpoint: Checkpoint, use_gpu: bool = False):
        ck = checkpoint if isinstance(checkpoint, GBDTCheckpoint) else GBDTCheckpoint(checkpoint.path)
        return cls(ck.get_model(), ck.get_preprocessor(), use_gpu)

    def predict(self, data, feature_columns: Optional[List[str]] = None, **predict_kwargs):
        import pandas as pd

        if self.preprocessor is not None:
            data = self.preprocessor.transform_batch(data)
        if isinstance(data, dict):
            data = pd.DataFrame(data)
        if isinstance(data, pd.DataFrame):
            cols = feature_columns or [c for c in (self.model.feature_names or data.columns) if c in data.columns]
            X = data[cols].to_numpy(dtype=np.float32, na_value=np.nan)
            import torch

            out = self.model.predict(torch.as_tensor(X, device=self.device), **predict_kwargs).cpu().numpy()
            if out.ndim == 2:
                return pd.DataFrame({f"predictions_{i}": out[:, i] for i in range(out.shape[1])})
            return pd.DataFrame({"predictions": out})
        arr = np.asarray(data, dtype=np.float32)
        if feature_columns is not None:
            arr = arr[:, feature_columns]
        return {"predictions": self.model.predict(arr, **predict_kwargs)}
