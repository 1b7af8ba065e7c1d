"""``ray.train.sklearn`` (reference: ``python/ray/train/sklearn/``): ``SklearnCheckpoint``,
``SklearnPredictor``; ``SklearnTrainer`` is deprecated there and raises the same way here
(``sklearn_trainer.py:14-35``: train sklearn models in a Tune trainable instead)."""
from __future__ import annotations

import os
import tempfile
from typing import List, Optional

import numpy as np

from .._checkpoint import Checkpoint

_DEPRECATION_MESSAGE = ("`ray.train.sklearn.SklearnTrainer` is deprecated. Write your own training loop instead "
                        "and use `ray.tune.Tuner` to parallelize the training of multiple sklearn models.")


class SklearnTrainer:
    def __new__(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION_MESSAGE)

    @classmethod
    def restore(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION_MESSAGE)

    @classmethod
    def can_restore(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION_MESSAGE)

    @staticmethod
    def get_model(*args, **kwargs):
        raise DeprecationWarning(_DEPRECATION_MESSAGE)


class SklearnCheckpoint(Checkpoint):
    """Checkpoint holding a fitted estimator (``model.pkl``, cloudpickle) and optionally a fitted
    preprocessor. Only load checkpoints you wrote yourself: unpickling runs code."""

    MODEL_FILENAME = "model.pkl"

    @classmethod
    def from_estimator(cls, estimator, *, path: Optional[str] = None, preprocessor=None) -> "SklearnCheckpoint":
        import cloudpickle

        path = path or tempfile.mkdtemp(prefix="rca_sklearn_ckpt_")
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, cls.MODEL_FILENAME), "wb") as f:
            cloudpickle.dump(estimator, f)
        if preprocessor is not None:
            with open(os.path.join(path, "preprocessor.pkl"), "wb") as f:
                cloudpickle.dump(preprocessor, f)
        return cls(path)

    def get_estimator(self):
        import cloudpickle

        with open(os.path.join(self.path, self.MODEL_FILENAME), "rb") as f:
            return cloudpickle.load(f)

    def get_preprocessor(self):
        p = os.path.join(self.path, "preprocessor.pkl")
        if not os.path.exists(p):
            return None
        import cloudpickle

        with open(p, "rb") as f:
            return cloudpickle.load(f)


def _set_cpu_params(estimator, num_cpus: int) -> None:
    """n_jobs / thread_count of the estimator and its nested estimators -> num_cpus."""
    try:
        params = estimator.get_params(deep=True)
    except Exception:  # not an sklearn estimator
        return
    upd = {k: num_cpus for k in params if k.endswith("n_jobs") or k.endswith("thread_count") or k == "nthread"}
    if upd:
        estimator.set_params(**upd)


class SklearnPredictor:
    """Batch inference with a fitted estimator: numpy / pandas / dict batches ->
    ``{"predictions": ...}`` (a DataFrame for DataFrame input, like the reference)."""

    def __init__(self, estimator, preprocessor=None):
        self.estimator = estimator
        self.preprocessor = preprocessor

    def __repr__(self):
        return f"SklearnPredictor(estimator={self.estimator!r}, preprocessor={self.preprocessor!r})"

    @classmethod
    def from_checkpoint(cls, checkpoint: Checkpoint) -> "SklearnPredictor":
        ck = checkpoint if isinstance(checkpoint, SklearnCheckpoint) else SklearnCheckpoint(checkpoint.path)
        return cls(ck.get_estimator(), ck.get_preprocessor())

    def get_preprocessor(self):
        return self.preprocessor

    def predict(self, data, feature_columns: Optional[List] = None, num_estimator_cpus: Optional[int] = None,
                **predict_kwargs):
        import pandas as pd

        if num_estimator_cpus:
            _set_cpu_params(self.estimator, num_estimator_cpus)
        if self.preprocessor is not None:
            data = self.preprocessor.transform_batch(data)
        if isinstance(data, dict):
            data = pd.DataFrame(data)
        if isinstance(data, pd.DataFrame):
            X = data[feature_columns] if feature_columns else data
            out = np.asarray(self.estimator.predict(X, **predict_kwargs))
            if out.ndim == 2:
                return pd.DataFrame({f"predictions_{i}": out[:, i] for i in range(out.shape[1])})
            return pd.DataFrame({"predictions": out})
        X = np.asarray(data)
        if feature_columns is not None:
            X = X[:, feature_columns]
        return {"predictions": np.asarray(self.estimator.predict(X, **predict_kwargs))}


__all__ = ["SklearnTrainer", "SklearnCheckpoint", "SklearnPredictor"]
