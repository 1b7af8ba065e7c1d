"""GroupedData (reference: ``python/ray/data/grouped_data.py``): hash-partitioned groupby."""
from __future__ import annotations

from typing import List, Optional, Union

from . import aggregate as A
from ._internal import execution as X


class GroupedData:
    def __init__(self, ds, key: Union[str, List[str], None]):
        self._ds = ds
        self._keys = [key] if isinstance(key, str) else (list(key) if key else [])

    def _shuffle(self, refs, **reduce_kw):
        k = max(1, min(len(refs), 16)) if self._keys else 1
        if self._keys:
            out = X.exchange(refs, k, X._split_by_hash, [(self._keys, k) for _ in refs], X._reduce_groupby,
                             [dict(keys=self._keys, **reduce_kw) for _ in range(k)])
        else:
            out = X.exchange(refs, 1, _all_in_one, [() for _ in refs], X._reduce_groupby,
                             [dict(keys=None, **reduce_kw)])
        return out

    def aggregate(self, *aggs: A.AggregateFn):
        from .dataset import Dataset

        def fn(refs):
            return self._shuffle(refs, aggs=list(aggs))

        ds = self._ds._with({"kind": "alltoall", "fn": fn})
        return ds.sort(list(self._keys)) if self._keys else ds  # grouped rows ordered by every key

    def count(self):
        return self.aggregate(A.Count())

    def sum(self, on=None, ignore_nulls=True):
        return self.aggregate(*[A.Sum(c) for c in _cols(on)])

    def min(self, on=None, ignore_nulls=True):
        return self.aggregate(*[A.Min(c) for c in _cols(on)])

    def max(self, on=None, ignore_nulls=True):
        return self.aggregate(*[A.Max(c) for c in _cols(on)])

    def mean(self, on=None, ignore_nulls=True):
        return self.aggregate(*[A.Mean(c) for c in _cols(on)])

    def std(self, on=None, ddof=1, ignore_nulls=True):
        return self.aggregate(*[A.Std(c, ddof=ddof) for c in _cols(on)])

    def map_groups(self, fn, *, batch_format: str = "default", compute=None, **kw):
        def f(refs):
            return self._shuffle(refs, map_groups=fn, batch_format="numpy" if batch_format == "default" else
                                 batch_format)

        return self._ds._with({"kind": "alltoall", "fn": f})


def _all_in_one(block):
    return [block]


def _aggregate_block(block, key, aggs):
    """One row per group of ``block`` (pandas groupby), each AggregateFn as a column; ``key`` None
    aggregates the whole block into one row."""
    import pandas as pd

    from .block import BlockAccessor, normalize_block

    df = BlockAccessor.for_block(block).to_pandas()
    keys = [key] if isinstance(key, str) else (list(key) if key else [])
    if not keys:
        return normalize_block(pd.DataFrame([{a.name: a.pandas_agg_all(df) for a in aggs}]))
    gb = df.groupby(keys, sort=True)
    out = pd.DataFrame({a.name: a.pandas_agg(gb) for a in aggs}).reset_index()
    return normalize_block(out)


def _cols(on):
    if on is None:
        raise ValueError("specify the column(s) to aggregate with on=")
    return [on] if isinstance(on, str) else list(on)
