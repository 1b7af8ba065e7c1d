"""Distributed iterators (reference: ``python/ray/util/iter.py``).

A ``ParallelIterator`` is a set of shard actors, each owning a Python iterator plus a lazily
applied transform chain (``for_each``/``filter``/``batch``/``flatten``). ``gather_sync`` pulls
from the shards round-robin in batches of ``batch_ms``-sized chunks; ``gather_async`` pulls from
whichever shard answers first. ``LocalIterator`` is the driver-side equivalent.
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, Iterable, Iterator, List, Optional

_END = "__rca_iter_end__"


def _apply(it: Iterator, ops: List):
    for kind, arg in ops:
        if kind == "for_each":
            it = map(arg, it)
        elif kind == "filter":
            it = filter(arg, it)
        elif kind == "batch":
            it = _batched(it, arg)
        elif kind == "flatten":
            it = (y for x in it for y in x)
    return it


def _batched(it, n):
    while True:
        b = list(itertools.islice(it, n))
        if not b:
            return
        yield b


class _Shard:
    def __init__(self, make_iter, repeat: bool):
        self._make = make_iter
        self._repeat = repeat
        self._ops: List = []
        self._it = None

    def set_ops(self, ops):
        self._ops = list(ops)
        self._it = None
        return True

    def _iter(self):
        if self._it is None:
            def gen():
                while True:
                    yield from self._make()
                    if not self._repeat:
                        return

            self._it = _apply(gen(), self._ops)
        return self._it

    def next_batch(self, n: int):
        out = list(itertools.islice(self._iter(), n))
        if len(out) < n:
            out.append(_END)
        return out


class LocalIterator:
    def __init__(self, base: Callable[[], Iterator], ops: Optional[List] = None, name: str = "LocalIterator"):
        self._base = base
        self._ops = list(ops or [])
        self.name = name

    def _derive(self, kind, arg, label):
        return LocalIterator(self._base, self._ops + [(kind, arg)], f"{self.name}.{label}")

    def for_each(self, fn):
        return self._derive("for_each", fn, "for_each()")

    def filter(self, fn):
        return self._derive("filter", fn, "filter()")

    def batch(self, n: int):
        return self._derive("batch", n, f"batch({n})")

    def flatten(self):
        return self._derive("flatten", None, "flatten()")

    def __iter__(self):
        return _apply(iter(self._base()), self._ops)

    def take(self, n: int) -> List:
        return list(itertools.islice(iter(self), n))

    def show(self, n: int = 20):
        for x in self.take(n):
            print(x)

    def union(self, *others: "LocalIterator") -> "LocalIterator":
        its = [self] + list(others)

        def base():
            gens = [iter(i) for i in its]
            while gens:
                for g in list(gens):
                    try:
                        yield next(g)
                    except StopIteration:
                        gens.remove(g)

        return LocalIterator(base, [], "LocalUnion")

    def __repr__(self):
        return f"LocalIterator[{self.name}]"


class ParallelIterator:
    def __init__(self, shards: List, ops: Optional[List] = None, name: str = "ParallelIterator", batch_size: int = 32):
        self._shards = shards
        self._ops = list(ops or [])
        self.name = name
        self._batch = batch_size

    def _derive(self, kind, arg, label):
        return ParallelIterator(self._shards, self._ops + [(kind, arg)], f"{self.name}.{label}", self._batch)

    def for_each(self, fn, max_concurrency: int = 1, resources=None):
        return self._derive("for_each", fn, "for_each()")

    def filter(self, fn):
        return self._derive("filter", fn, "filter()")

    def batch(self, n: int):
        return self._derive("batch", n, f"batch({n})")

    def flatten(self):
        return self._derive("flatten", None, "flatten()")

    def num_shards(self) -> int:
        return len(self._shards)

    def shards(self) -> List[LocalIterator]:
        return [self.get_shard(i) for i in range(len(self._shards))]

    def get_shard(self, i: int) -> LocalIterator:
        from .._private.worker import get

        shard, ops, b = self._shards[i], self._ops, self._batch

        def base():
            get(shard.set_ops.remote(ops))
            while True:
                items = get(shard.next_batch.remote(b))
                for x in items:
                    if isinstance(x, str) and x == _END:
                        return
                    yield x

        return LocalIterator(base, [], f"{self.name}.shard[{i}]")

    def gather_sync(self) -> LocalIterator:
        from .._private.worker import get

        shards, ops, b = self._shards, self._ops, self._batch

        def base():
            get([s.set_ops.remote(ops) for s in shards])
            live = list(shards)
            while live:
                outs = get([s.next_batch.remote(b) for s in live])
                nxt = []
                for s, items in zip(live, outs):
                    ended = False
                    for x in items:
                        if isinstance(x, str) and x == _END:
                            ended = True
                            break
                        yield x
                    if not ended:
                        nxt.append(s)
                live = nxt

        return LocalIterator(base, [], f"{self.name}.gather_sync()")

    def gather_async(self, batch_ms: int = 0, num_async: int = 1) -> LocalIterator:
        from .._private.worker import get, wait

        shards, ops, b = self._shards, self._ops, self._batch

        def base():
            get([s.set_ops.remote(ops) for s in shards])
            pending = {s.next_batch.remote(b): s for s in shards}
            while pending:
                ready, _ = wait(list(pending), num_returns=1)
                for ref in ready:
                    s = pending.pop(ref)
                    ended = False
                    for x in get(ref):
                        if isinstance(x, str) and x == _END:
                            ended = True
                            break
                        yield x
                    if not ended:
                        pending[s.next_batch.remote(b)] = s

        return LocalIterator(base, [], f"{self.name}.gather_async()")

    def union(self, other: "ParallelIterator") -> "ParallelIterator":
        if self._ops or other._ops:
            raise ValueError("union() of transformed ParallelIterators is not supported; union first")
        return ParallelIterator(self._shards + other._shards, [], f"ParallelUnion[{self.name}, {other.name}]",
                                self._batch)

    def take(self, n: int) -> List:
        return self.gather_sync().take(n)

    def show(self, n: int = 20):
        self.gather_sync().show(n)

    def __iter__(self):
        raise TypeError("You must use it.gather_sync() or it.gather_async() to iterate over a ParallelIterator.")

    def __repr__(self):
        return f"ParallelIterator[{self.name}]"


def _make_shards(factories, repeat):
    from ..actor import ActorClass

    cls = ActorClass(_Shard, {"num_cpus": 0})
    return [cls.remote(f, repeat) for f in factories]


def from_items(items: List[Any], num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    items = list(items)
    parts = [items[i::num_shards] for i in range(num_shards)]
    shards = _make_shards([(lambda p=p: iter(p)) for p in parts], repeat)
    return ParallelIterator(shards, [], f"from_items[{type(items[0]).__name__ if items else 'Any'}, "
                                        f"{len(items)}, shards={num_shards}]")


def from_range(n: int, num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    per = (n + num_shards - 1) // num_shards
    bounds = [(i * per, min(n, (i + 1) * per)) for i in range(num_shards)]
    shards = _make_shards([(lambda a=a, b=b: iter(range(a, b))) for a, b in bounds], repeat)
    return ParallelIterator(shards, [], f"from_range[{n}, shards={num_shards}]")


def from_iterators(generators: List[Iterable], repeat: bool = False, name=None) -> ParallelIterator:
    facs = []
    for g in generators:
        if callable(g):
            facs.append(g)
        else:
            data = list(g)
            facs.append(lambda d=data: iter(d))
    return ParallelIterator(_make_shards(facs, repeat), [], name or f"from_iterators[shards={len(facs)}]")


def from_actors(actors: List, name=None) -> ParallelIterator:
    return ParallelIterator(list(actors), [], name or f"from_actors[shards={len(actors)}]")
