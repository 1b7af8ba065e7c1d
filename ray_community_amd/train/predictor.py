"""Predictor base (reference: python/ray/train/predictor.py): a model + optional preprocessor
that maps a batch to predictions. ``TorchPredictor``, ``SklearnPredictor`` and the GBDT
predictors follow this interface."""
from __future__ import annotations

from typing import Any, Optional


class PredictorNotSerializableException(RuntimeError):
    """Predictors hold live models; build them in each worker from a checkpoint instead."""


class Predictor:
    def __init__(self, preprocessor=None):
        self._preprocessor = preprocessor

    @classmethod
    def from_checkpoint(cls, checkpoint, **kwargs) -> "Predictor":
        raise NotImplementedError

    @classmethod
    def from_pandas_udf(cls, pandas_udf):
        """A Predictor whose ``predict`` runs ``pandas_udf(df) -> df``."""
        class _UDF(Predictor):
            def _predict_pandas(self, df, **kw):
                return pandas_udf(df, **kw)
        return _UDF()

    def get_preprocessor(self):
        return self._preprocessor

    def set_preprocessor(self, preprocessor) -> None:
        self._preprocessor = preprocessor

    @classmethod
    def preferred_batch_format(cls) -> str:
        return "pandas"

    def predict(self, data: Any, **kwargs):
        import pandas as pd

        if self._preprocessor is not None:
            data = self._preprocessor.transform_batch(data)
        df = data if isinstance(data, pd.DataFrame) else pd.DataFrame(data)
        return self._predict_pandas(df, **kwargs)

    def _predict_pandas(self, df, **kwargs):
        raise NotImplementedError

    def __reduce__(self):
        raise PredictorNotSerializableException(
            f"{type(self).__name__} is not serializable; create it from a checkpoint where it is used")
