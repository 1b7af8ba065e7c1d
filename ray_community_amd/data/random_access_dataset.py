"""Key-value lookups over a sorted Dataset (reference: ``python/ray/data/random_access_dataset.py``).

``Dataset.to_random_access_dataset(key, num_workers)`` sorts by ``key``, deals the sorted blocks
to ``num_workers`` actors in contiguous ranges and keeps each actor's first key on the caller:
``get_async(k)`` bisects that table and asks one actor, which binary-searches its key array
(one ``np.searchsorted`` per lookup, rows materialised only on a hit); ``multiget`` groups keys by
actor so each actor is asked once.
"""
from __future__ import annotations

import bisect
from typing import Any, List, Optional

import numpy as np

from .block import BlockAccessor, concat_blocks


class _Shard:
    def __init__(self, key: str, blocks):
        from .._private.worker import get

        bl = [get(b) for b in blocks]
        bl = [b for b in bl if BlockAccessor(b).num_rows()]
        self.block = concat_blocks(bl) if bl else None
        self.cols = BlockAccessor(self.block).to_numpy() if self.block is not None else {}
        self.keys = self.cols.get(key, np.asarray([]))
        self.hits = 0

    def first_key(self):
        return self.keys[0] if len(self.keys) else None

    def _row(self, i):
        return {c: (v[i].item() if isinstance(v[i], np.generic) else v[i]) for c, v in self.cols.items()}

    def get(self, k):
        i = int(np.searchsorted(self.keys, k))
        if i < len(self.keys) and self.keys[i] == k:
            self.hits += 1
            return self._row(i)
        return None

    def multiget(self, ks):
        return [self.get(k) for k in ks]

    def stats(self):
        return {"num_rows": int(len(self.keys)), "hits": self.hits}


class RandomAccessDataset:
    def __init__(self, ds, key: str, num_workers: int):
        from ..actor import ActorClass
        from .._private.worker import get

        sorted_ds = ds.sort(key).materialize()
        refs = [b for b, _ in sorted_ds._refs()]
        n = max(1, min(num_workers, len(refs)))
        cls = ActorClass(_Shard, {"num_cpus": 0})
        self._workers = [cls.remote(key, refs[len(refs) * i // n: len(refs) * (i + 1) // n]) for i in range(n)]
        firsts = get([w.first_key.remote() for w in self._workers])
        keep = [(f, w) for f, w in zip(firsts, self._workers) if f is not None]
        self._lower = [f for f, _ in keep]
        self._live = [w for _, w in keep]
        self.key = key

    def _owner(self, k) -> Optional[int]:
        i = bisect.bisect_right(self._lower, k) - 1
        return i if i >= 0 else None

    def get_async(self, key: Any):
        """ObjectRef of the row whose key equals ``key`` (None when there is none)."""
        from .._private.worker import put

        i = self._owner(key)
        if i is None:
            return put(None)
        return self._live[i].get.remote(key)

    def multiget(self, keys: List[Any]) -> List[Optional[dict]]:
        from .._private.worker import get

        by = {}
        for pos, k in enumerate(keys):
            i = self._owner(k)
            if i is not None:
                by.setdefault(i, []).append((pos, k))
        out: List[Optional[dict]] = [None] * len(keys)
        refs = {i: self._live[i].multiget.remote([k for _, k in items]) for i, items in by.items()}
        for i, items in by.items():
            for (pos, _), row in zip(items, get(refs[i])):
                out[pos] = row
        return out

    def stats(self) -> str:
        from .._private.worker import get

        st = get([w.stats.remote() for w in self._live])
        return "RandomAccessDataset:\n" + "\n".join(
            f"  worker {i}: {s['num_rows']} rows, {s['hits']} hits" for i, s in enumerate(st))
