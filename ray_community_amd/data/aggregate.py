"""Aggregations (reference: ``python/ray/data/aggregate``)."""
from __future__ import annotations

from typing import Callable, Optional


class AggregateFn:
    """A built-in aggregation (``how``) over column ``on``, or -- reference form
    ``AggregateFn(init, merge, name, accumulate_row=..., accumulate_block=..., finalize=...)`` -- a
    user-defined one: per group ``acc = init(key)``, then ``accumulate_block(acc, block)`` (a pandas
    DataFrame of the group) or ``accumulate_row(acc, row)`` per row, and ``finalize(acc)``. Every
    group is reduced in one place after the hash exchange, so ``merge`` is not needed to combine
    partials here (it is accepted for API compatibility)."""

    def __init__(self, on=None, alias_name: Optional[str] = None, how: str = "sum", ddof: int = 1,
                 ignore_nulls: bool = True, *, init: Optional[Callable] = None, merge: Optional[Callable] = None,
                 name: Optional[str] = None, accumulate_row: Optional[Callable] = None,
                 accumulate_block: Optional[Callable] = None, finalize: Optional[Callable] = None,
                 q: float = 0.5):
        if callable(on) and init is None:  # AggregateFn(init, merge, name, ...) positionally
            init, merge, name, on = on, alias_name if callable(alias_name) else merge, \
                (how if how != "sum" else name), None
            alias_name = None
        self.init, self.merge, self.finalize = init, merge, finalize
        self.accumulate_row, self.accumulate_block = accumulate_row, accumulate_block
        if init is not None:
            if accumulate_row is None and accumulate_block is None:
                raise ValueError("a custom AggregateFn needs accumulate_row or accumulate_block")
            how = "custom"
        self.on = on
        self.how = how
        self.ddof = ddof
        self.q = q
        self.ignore_nulls = ignore_nulls
        self.name = name or alias_name or (f"{how}({on})" if on else f"{how}()")

    def _custom(self, key, df):
        acc = self.init(key)
        if self.accumulate_block is not None:
            acc = self.accumulate_block(acc, df.reset_index(drop=True))
        else:
            for row in df.to_dict("records"):
                acc = self.accumulate_row(acc, row)
        return self.finalize(acc) if self.finalize is not None else acc

    def pandas_agg(self, gb):
        if self.how == "custom":
            import pandas as pd

            vals = [self._custom(k[0] if isinstance(k, tuple) and len(k) == 1 else k, g) for k, g in gb]
            return pd.Series(vals, index=gb.size().index, dtype=object)  # groups iterate in index order
        if self.how == "quantile":
            return gb[self.on].quantile(self.q)
        if self.how == "count":
            return gb.size()
        col = gb[self.on]
        if self.how == "std":
            return col.std(ddof=self.ddof)
        if self.how == "absmax":
            return col.apply(lambda s: s.abs().max())
        if self.how == "unique":
            return col.apply(lambda s: list(s.unique()))
        return getattr(col, self.how)()

    def pandas_agg_all(self, df):
        if self.how == "custom":
            return self._custom(None, df)
        if self.how == "quantile":
            return df[self.on].quantile(self.q)
        if self.how == "count":
            return len(df)
        s = df[self.on]
        if self.how == "std":
            return s.std(ddof=self.ddof)
        if self.how == "absmax":
            return s.abs().max()
        if self.how == "unique":
            return list(s.unique())
        return getattr(s, self.how)()


class Count(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name or "count()", "count")


class Sum(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "sum")


class Min(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "min")


class Max(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "max")


class Mean(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "mean")


class Std(AggregateFn):
    def __init__(self, on=None, ddof=1, alias_name=None, **kw):
        super().__init__(on, alias_name, "std", ddof=ddof)


class AbsMax(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "absmax")


class Unique(AggregateFn):
    def __init__(self, on=None, alias_name=None, **kw):
        super().__init__(on, alias_name, "unique")


class Quantile(AggregateFn):
    """The ``q`` quantile of column ``on`` (linear interpolation, as pandas / numpy)."""

    def __init__(self, on=None, q: float = 0.5, ignore_nulls: bool = True, alias_name=None, **kw):
        if not 0.0 <= q <= 1.0:
            raise ValueError("q must be in [0, 1]")
        super().__init__(on, alias_name or f"quantile({on})", "quantile", q=q, ignore_nulls=ignore_nulls)
