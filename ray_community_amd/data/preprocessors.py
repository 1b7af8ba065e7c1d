"""Preprocessors (reference: ``python/ray/data/preprocessors``)."""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np


class PreprocessorNotFittedException(RuntimeError):
    """``transform`` on a fittable preprocessor that was never fitted."""


class Preprocessor:
    _is_fittable = True

    class FitStatus(str):
        NOT_FITTABLE = "NOT_FITTABLE"
        NOT_FITTED = "NOT_FITTED"
        PARTIALLY_FITTED = "PARTIALLY_FITTED"  # a Chain with some fitted stages
        FITTED = "FITTED"

    def __init__(self):
        self.stats_: Optional[Dict] = None

    def fit_status(self) -> str:
        if not self._is_fittable:
            return Preprocessor.FitStatus.NOT_FITTABLE
        return Preprocessor.FitStatus.FITTED if self.stats_ is not None else Preprocessor.FitStatus.NOT_FITTED

    @classmethod
    def preferred_batch_format(cls) -> str:
        return "pandas"

    def serialize(self) -> str:
        """A string form of this preprocessor (fitted state included); ``deserialize`` restores it."""
        import base64

        import cloudpickle

        return base64.b64encode(cloudpickle.dumps(self)).decode("ascii")

    @staticmethod
    def deserialize(serialized: str) -> "Preprocessor":
        import base64
        import pickle

        return pickle.loads(base64.b64decode(serialized))  # a string produced by serialize()

    def fit(self, ds) -> "Preprocessor":
        if self._is_fittable:
            self.stats_ = self._fit(ds)
        return self

    def fit_transform(self, ds):
        return self.fit(ds).transform(ds)

    def transform(self, ds):
        if self._is_fittable and self.stats_ is None:
            raise PreprocessorNotFittedException(f"`{type(self).__name__}` must be fitted before transform")
        return ds.map_batches(self._transform_pandas, batch_format="pandas")

    def transform_batch(self, batch):
        import pandas as pd

        if self._is_fittable and self.stats_ is None:
            raise PreprocessorNotFittedException(f"`{type(self).__name__}` must be fitted before transform_batch")
        is_df = isinstance(batch, pd.DataFrame)
        df = batch if is_df else pd.DataFrame({k: list(v) if np.ndim(v) > 1 else v for k, v in batch.items()})
        out = self._transform_pandas(df)
        if is_df:
            return out
        return {c: np.stack(out[c].to_numpy()) if len(out) and isinstance(out[c].iloc[0], np.ndarray)
                else out[c].to_numpy() for c in out.columns}  # the batch format it was given

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


# ------------------------------------------------------------------------- more preprocessors
# (reference: python/ray/data/preprocessors/{scaler,normalizer,transformer,encoder,hasher,
# vectorizer,tokenizer,discretizer,torch}.py -- same constructor arguments and output semantics)
class RobustScaler(Preprocessor):
    """(x - median) / (q_high - q_low) with ``quantile_range`` percent quantiles."""

    def __init__(self, columns: List[str], quantile_range=(0.25, 0.75)):
        super().__init__()
        self.columns, self.quantile_range = columns, quantile_range

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        lo, hi = self.quantile_range
        return {c: (float(df[c].quantile(0.5)), float(df[c].quantile(lo)), float(df[c].quantile(hi)))
                for c in self.columns}

    def _transform_pandas(self, df):
        for c in self.columns:
            med, ql, qh = self.stats_[c]
            df[c] = (df[c] - med) / ((qh - ql) if qh != ql else 1.0)
        return df


class Normalizer(Preprocessor):
    """Scales each ROW of ``columns`` to unit ``norm`` ("l1", "l2" or "max")."""
    _is_fittable = False

    def __init__(self, columns: List[str], norm: str = "l2"):
        super().__init__()
        if norm not in ("l1", "l2", "max"):
            raise ValueError(f"norm must be l1, l2 or max, got {norm!r}")
        self.columns, self.norm = columns, norm

    def _transform_pandas(self, df):
        x = df[self.columns].to_numpy(dtype=np.float64)
        n = {"l1": np.abs(x).sum(1), "l2": np.sqrt((x * x).sum(1)), "max": np.abs(x).max(1)}[self.norm]
        n[n == 0] = 1.0
        df[self.columns] = x / n[:, None]
        return df


class PowerTransformer(Preprocessor):
    """Yeo-Johnson or Box-Cox with a fixed ``power`` (the reference's semantics; no lambda fit)."""
    _is_fittable = False

    def __init__(self, columns: List[str], power: float, method: str = "yeo-johnson"):
        super().__init__()
        if method not in ("yeo-johnson", "box-cox"):
            raise ValueError(f"unknown method {method!r}")
        self.columns, self.power, self.method = columns, power, method

    def _transform_pandas(self, df):
        p = self.power
        for c in self.columns:
            x = df[c].to_numpy(dtype=np.float64)
            if self.method == "box-cox":
                y = np.log(x) if p == 0 else (np.power(x, p) - 1) / p
            else:
                y = np.empty_like(x)
                pos = x >= 0
                y[pos] = np.log1p(x[pos]) if p == 0 else (np.power(x[pos] + 1, p) - 1) / p
                y[~pos] = (-np.log1p(-x[~pos]) if p == 2 else
                           -(np.power(-x[~pos] + 1, 2 - p) - 1) / (2 - p))
            df[c] = y
        return df


class Categorizer(Preprocessor):
    """Converts columns to pandas ``category`` dtype with the categories seen in ``fit``."""

    def __init__(self, columns: List[str], dtypes: Optional[Dict] = None):
        super().__init__()
        self.columns, self.dtypes = columns, dtypes or {}
        if self.dtypes and set(self.dtypes) >= set(columns):
            self._is_fittable = False

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        return {c: sorted(df[c].dropna().unique().tolist()) for c in self.columns if c not in self.dtypes}

    def _transform_pandas(self, df):
        import pandas as pd

        for c in self.columns:
            dt = self.dtypes.get(c) or pd.CategoricalDtype((self.stats_ or {}).get(c, []))
            df[c] = df[c].astype(dt)
        return df


class MultiHotEncoder(Preprocessor):
    """List-valued columns -> fixed-length count vectors over the categories seen in ``fit``."""

    def __init__(self, columns: List[str], *, max_categories: Optional[Dict[str, int]] = None):
        super().__init__()
        self.columns, self.max_categories = columns, max_categories or {}

    def _fit(self, ds):
        from collections import Counter

        df = ds.select_columns(self.columns).to_pandas()
        out = {}
        for c in self.columns:
            cnt = Counter(v for lst in df[c] for v in (lst if isinstance(lst, (list, tuple, np.ndarray)) else [lst]))
            cats = [k for k, _ in cnt.most_common(self.max_categories.get(c))]
            out[c] = {k: i for i, k in enumerate(sorted(cats, key=str))}
        return out

    def _transform_pandas(self, df):
        for c in self.columns:
            idx = self.stats_[c]

            def enc(lst, idx=idx):
                v = np.zeros(len(idx), dtype=np.int64)
                for x in (lst if isinstance(lst, (list, tuple, np.ndarray)) else [lst]):
                    j = idx.get(x)
                    if j is not None:
                        v[j] += 1
                return v

            df[c] = df[c].map(enc)
        return df


def _stable_hash(s: str, n: int) -> int:
    import zlib

    return zlib.crc32(str(s).encode()) % n


class FeatureHasher(Preprocessor):
    """Hashes the (token -> count) columns into ``num_features`` buckets: ``hash_{i}`` columns."""
    _is_fittable = False

    def __init__(self, columns: List[str], num_features: int):
        super().__init__()
        self.columns, self.num_features = columns, num_features

    def _transform_pandas(self, df):
        m = np.zeros((len(df), self.num_features))
        for c in self.columns:
            j = _stable_hash(c, self.num_features)
            m[:, j] += df[c].to_numpy(dtype=np.float64)
        df = df.drop(columns=self.columns)
        for j in range(self.num_features):
            df[f"hash_{j}"] = m[:, j]
        return df


def _split_tokens(s: str) -> List[str]:
    return str(s).split()


class Tokenizer(Preprocessor):
    """Replaces each string with its list of tokens (``tokenization_fn``, default whitespace split)."""
    _is_fittable = False

    def __init__(self, columns: List[str], tokenization_fn: Optional[Callable[[str], List[str]]] = None):
        super().__init__()
        self.columns, self.fn = columns, tokenization_fn or _split_tokens

    def _transform_pandas(self, df):
        for c in self.columns:
            df[c] = df[c].map(self.fn)
        return df


class HashingVectorizer(Preprocessor):
    """Token counts hashed into ``num_features`` columns ``hash_{col}_{i}`` per input column."""
    _is_fittable = False

    def __init__(self, columns: List[str], num_features: int, tokenization_fn=None):
        super().__init__()
        self.columns, self.num_features, self.fn = columns, num_features, tokenization_fn or _split_tokens

    def _transform_pandas(self, df):
        for c in self.columns:
            m = np.zeros((len(df), self.num_features), dtype=np.int64)
            for i, s in enumerate(df[c]):
                for tok in self.fn(s):
                    m[i, _stable_hash(tok, self.num_features)] += 1
            df = df.drop(columns=[c])
            for j in range(self.num_features):
                df[f"hash_{c}_{j}"] = m[:, j]
        return df


class CountVectorizer(Preprocessor):
    """Counts of the ``max_features`` most frequent tokens seen in ``fit``: columns ``{col}_{token}``."""

    def __init__(self, columns: List[str], tokenization_fn=None, max_features: Optional[int] = None):
        super().__init__()
        self.columns, self.fn, self.max_features = columns, tokenization_fn or _split_tokens, max_features

    def _fit(self, ds):
        from collections import Counter

        df = ds.select_columns(self.columns).to_pandas()
        return {c: [t for t, _ in Counter(t for s in df[c] for t in self.fn(s)).most_common(self.max_features)]
                for c in self.columns}

    def _transform_pandas(self, df):
        from collections import Counter

        for c in self.columns:
            counts = [Counter(self.fn(s)) for s in df[c]]
            vocab = self.stats_[c]
            df = df.drop(columns=[c])
            for tok in vocab:
                df[f"{c}_{tok}"] = [cn.get(tok, 0) for cn in counts]
        return df


class CustomKBinsDiscretizer(Preprocessor):
    """Bins values with explicit ``bins`` edges (a list, or a per-column dict); ``right`` /
    ``include_lowest`` as ``pandas.cut``; values are replaced by their bin index."""
    _is_fittable = False

    def __init__(self, columns: List[str], bins, *, right: bool = True, include_lowest: bool = False,
                 duplicates: str = "raise", dtypes: Optional[Dict] = None):
        super().__init__()
        self.columns, self.bins, self.right = columns, bins, right
        self.include_lowest, self.duplicates, self.dtypes = include_lowest, duplicates, dtypes

    def _edges(self, c):
        return self.bins[c] if isinstance(self.bins, dict) else self.bins

    def _transform_pandas(self, df):
        import pandas as pd

        for c in self.columns:
            df[c] = pd.cut(df[c], self._edges(c), right=self.right, include_lowest=self.include_lowest,
                           duplicates=self.duplicates, labels=False)
        return df


class UniformKBinsDiscretizer(CustomKBinsDiscretizer):
    """``bins`` equal-width bins between each column's min and max seen in ``fit``."""
    _is_fittable = True

    def __init__(self, columns: List[str], bins, *, right: bool = True, include_lowest: bool = False,
                 duplicates: str = "raise", dtypes: Optional[Dict] = None):
        super().__init__(columns, bins, right=right, include_lowest=include_lowest, duplicates=duplicates,
                         dtypes=dtypes)
        self._is_fittable = True

    def _fit(self, ds):
        df = ds.select_columns(self.columns).to_pandas()
        out = {}
        for c in self.columns:
            k = self.bins[c] if isinstance(self.bins, dict) else self.bins
            out[c] = np.linspace(float(df[c].min()), float(df[c].max()), int(k) + 1).tolist()
        return out

    def _edges(self, c):
        return self.stats_[c]


class TorchVisionPreprocessor(Preprocessor):
    """Applies a (torchvision-style) callable to each image in ``columns`` (``batched=True``: to the
    whole stacked batch); outputs go to ``output_columns`` (default: in place)."""
    _is_fittable = False

    def __init__(self, columns: List[str], transform: Callable, output_columns: Optional[List[str]] = None,
                 batched: bool = False):
        super().__init__()
        self.columns, self.transform_fn, self.batched = columns, transform, batched
        self.output_columns = output_columns or columns

    def transform(self, ds):
        return ds.map_batches(self._transform_numpy, batch_format="numpy")

    def transform_batch(self, batch):
        return self._transform_numpy(dict(batch))

    def _apply(self, arr):
        import torch

        t = torch.as_tensor(np.ascontiguousarray(arr))
        if self.batched:
            out = self.transform_fn(t)
        else:
            out = torch.stack([torch.as_tensor(self.transform_fn(x)) for x in t])
        return out.numpy() if isinstance(out, torch.Tensor) else np.asarray(out)

    def _transform_numpy(self, batch):
        for c, o in zip(self.columns, self.output_columns):
            batch[o] = self._apply(batch[c])
        return batch
