"""Aggregations (reference: ``python/ray/data/aggregate``)."""
from __future__ import annotations

from typing import Optional


class AggregateFn:
    def __init__(self, on: Optional[str] = None, alias_name: Optional[str] = None, how: str = "sum", ddof: int = 1,
                 ignore_nulls: bool = True):
        self.on = on
        self.how = how
        self.ddof = ddof
        self.name = alias_name or (f"{how}({on})" if on else f"{how}()")

    def pandas_agg(self, gb):
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
