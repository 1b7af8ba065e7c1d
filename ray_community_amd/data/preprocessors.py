"""Preprocessors (reference: ``python/ray/data/preprocessors``)."""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np


class Preprocessor:
    _is_fittable = True

    def __init__(self):
        self.stats_: Optional[Dict] = None

    def fit(self, ds) -> "Preprocessor":
        if self._is_fittable:
            self.stats_ = self._fit(ds)
        return self

    def fit_transform(self, ds):
        return self.fit(ds).transform(ds)

    def transform(self, ds):
        if self._is_fittable and self.stats_ is None:
            raise RuntimeError(f"`{type(self).__name__}` must be fitted before transform")
        return ds.map_batches(self._transform_pandas, batch_format="pandas")

    def transform_batch(self, batch):
        import pandas as pd

        df = batch if isinstance(batch, pd.DataFrame) else pd.DataFrame({k: list(v) if np.ndim(v) > 1 else v
                                                                        for k, v in batch.items()})
        return self._transform_pandas(df)

    def _fit(self, ds) -> Dict:
        return {}

    def _transform_pandas(self, df):
        raise NotImplementedError


class StandardScaler(Preprocessor):
    def __init__(self, columns: List[str], ddof: int = 0):
        super().__init__()
        self.columns = columns
        self.ddof = ddof

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        return {c: (float(df[c].mean()), float(df[c].std(ddof=self.ddof))) for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            m, s = self.stats_[c]
            df[c] = (df[c] - m) / (s if s else 1.0)
        return df


class MinMaxScaler(Preprocessor):
    def __init__(self, columns: List[str]):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        return {c: (float(df[c].min()), float(df[c].max())) for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            lo, hi = self.stats_[c]
            df[c] = (df[c] - lo) / ((hi - lo) if hi > lo else 1.0)
        return df


class MaxAbsScaler(Preprocessor):
    def __init__(self, columns: List[str]):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        return {c: float(df[c].abs().max()) for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            m = self.stats_[c]
            df[c] = df[c] / (m if m else 1.0)
        return df


class LabelEncoder(Preprocessor):
    def __init__(self, label_column: str):
        super().__init__()
        self.label_column = label_column

    def _fit(self, ds):
        vals = sorted(ds.unique(self.label_column))
        return {"classes": {v: i for i, v in enumerate(vals)}}

    def _transform_pandas(self, df):
        df[self.label_column] = df[self.label_column].map(self.stats_["classes"])
        return df

    def inverse_transform_batch(self, df):
        inv = {i: v for v, i in self.stats_["classes"].items()}
        df[self.label_column] = df[self.label_column].map(inv)
        return df


class OrdinalEncoder(Preprocessor):
    def __init__(self, columns: List[str]):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        return {c: {v: i for i, v in enumerate(sorted(ds.unique(c)))} for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            df[c] = df[c].map(self.stats_[c])
        return df


class OneHotEncoder(Preprocessor):
    def __init__(self, columns: List[str], max_categories: Optional[Dict[str, int]] = None):
        super().__init__()
        self.columns = columns

    def _fit(self, ds):
        return {c: sorted(ds.unique(c)) for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            cats = self.stats_[c]
            for v in cats:
                df[f"{c}_{v}"] = (df[c] == v).astype(np.int64)
            df = df.drop(columns=[c])
        return df


class SimpleImputer(Preprocessor):
    def __init__(self, columns: List[str], strategy: str = "mean", fill_value=None):
        super().__init__()
        self.columns = columns
        self.strategy = strategy
        self.fill_value = fill_value
        self._is_fittable = strategy != "constant"

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        if self.strategy == "mean":
            return {c: float(df[c].mean()) for c in self.columns}
        if self.strategy == "most_frequent":
            return {c: df[c].mode().iloc[0] for c in self.columns}
        return {}

    def _transform_pandas(self, df):
        for c in self.columns:
            v = self.fill_value if self.strategy == "constant" else self.stats_[c]
            df[c] = df[c].fillna(v)
        return df


class Concatenator(Preprocessor):
    _is_fittable = False

    def __init__(self, output_column_name: str = "concat_out", include: Optional[List[str]] = None,
                 exclude: Optional[List[str]] = None, dtype=np.float32, columns=None):
        super().__init__()
        self.out = output_column_name
        self.include = include or columns
        self.exclude = exclude or []
        self.dtype = dtype

    def transform(self, ds):
        return ds.map_batches(self._np, batch_format="numpy")

    def _np(self, batch):
        cols = [c for c in (self.include or list(batch)) if c not in self.exclude]
        arr = np.stack([np.asarray(batch[c], dtype=self.dtype).reshape(len(batch[c]), -1) for c in cols],
                       axis=1).reshape(len(batch[cols[0]]), -1)
        out = {k: v for k, v in batch.items() if k not in cols}
        out[self.out] = arr
        return out

    def _transform_pandas(self, df):
        d = {c: df[c].to_numpy() for c in df.columns}
        return self._np(d)


class BatchMapper(Preprocessor):
    _is_fittable = False

    def __init__(self, fn: Callable, batch_format: str = "pandas", batch_size=None):
        super().__init__()
        self.fn = fn
        self.batch_format = batch_format

    def transform(self, ds):
        return ds.map_batches(self.fn, batch_format=self.batch_format)

    def _transform_pandas(self, df):
        return self.fn(df)


class Chain(Preprocessor):
    def __init__(self, *preprocessors: Preprocessor):
        super().__init__()
        self.preprocessors = preprocessors

    def fit(self, ds):
        for p in self.preprocessors:
            ds = p.fit_transform(ds) if p._is_fittable else p.transform(ds)
        self.stats_ = {}
        return self

    def transform(self, ds):
        for p in self.preprocessors:
            ds = p.transform(ds)
        return ds

    def transform_batch(self, batch):
        for p in self.preprocessors:
            batch = p.transform_batch(batch)
        return batch
