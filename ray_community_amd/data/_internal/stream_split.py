"""Streaming split: one execution of a Dataset feeding ``n`` consumers lazily (reference:
``python/ray/data/dataset.py:1141`` ``streaming_split``,
``_internal/iterator/stream_split_iterator.py:32`` ``StreamSplitDataIterator`` / ``:128``
``SplitCoordinator``, ``_internal/execution/operators/output_splitter.py`` ``OutputSplitter``).

A ``SplitCoordinator`` actor owns the execution. Each consumer's ``StreamSplitDataIterator`` opens
an epoch with ``start_epoch`` -- a barrier: the dataset is (re-)executed only once all ``n``
consumers have asked for the epoch, so a ``random_shuffle`` (unseeded) gives a fresh order every
epoch -- then pulls block refs with ``get``. The coordinator runs the streaming executor in its own
process and routes output blocks as they come:

* ``equal=False``: a block goes to the consumer whose request pulled it (dynamic load balancing:
  a fast consumer takes more blocks), or, with ``locality_hints``, to a requester on the block's
  node when one is waiting;
* ``equal=True``: blocks go to the consumer with the fewest rows so far, from a hold-back buffer
  of at least ``n * (max block rows + 1)`` rows; at the end of the stream the buffer is cut (slice
  tasks) so every consumer gets exactly ``total // n`` rows (the remainder is dropped, as in the
  reference).

Blocks are referenced only by the consumer that receives them, so a dataset larger than the
object store streams through: the executor's output window bounds what is in flight.
"""
from __future__ import annotations

import collections
import itertools
import threading
import time
from typing import Any, List, Optional

from ..iterator import DataIterator

_POLL_S = 0.05


class SplitCoordinator:
    def __init__(self, ds, n: int, equal: bool, locality_hints: Optional[List[Any]]):
        self._ds = ds
        self._n = n
        self._equal = equal
        self._hints = list(locality_hints) if locality_hints else None
        self._cv = threading.Condition()
        self._epoch = -1
        self._split_epoch = [-1] * n
        self._arrived = collections.defaultdict(set)
        self._queues = [collections.deque() for _ in range(n)]
        self._turn = [0] * n  # per consumer: seq of the get() call answered next
        self._it = None
        self._done = True
        self._pulling = False
        self._buffer = collections.deque()  # equal mode hold-back: (block, meta, rows)
        self._buffer_rows = 0
        self._assigned = [0] * n
        self._max_rows = 0
        self._stats = {"epochs": 0, "blocks": [0] * n, "rows": [0] * n}

    # ---------------------------------------------------------------- epochs
    def start_epoch(self, split_idx: int) -> int:
        with self._cv:
            e = self._split_epoch[split_idx] + 1
            self._split_epoch[split_idx] = e
            self._arrived[e].add(split_idx)
            if len(self._arrived[e]) == self._n:
                self._begin(e)
                self._cv.notify_all()
            while self._epoch < e:
                self._cv.wait(_POLL_S)
            return e

    def _begin(self, e: int):
        self._arrived.pop(e, None)
        self._epoch = e
        self._queues = [collections.deque() for _ in range(self._n)]
        self._turn = [0] * self._n
        self._buffer.clear()
        self._buffer_rows = 0
        self._assigned = [0] * self._n
        self._max_rows = 0
        self._done = False
        self._it = self._ds._iter_refs()  # a fresh streaming execution of the plan
        self._stats["epochs"] += 1

    # ---------------------------------------------------------------- blocks
    def get(self, epoch: int, split_idx: int, seq: int = 0):
        """The ``seq``-th ``[block_ref, meta_ref]`` of this consumer in ``epoch``, or None at its
        end. A consumer keeps several calls in flight (prefetch) and reads their replies in
        order, so the calls are answered in ``seq`` order whatever order they run in."""
        while True:
            with self._cv:
                while True:
                    if epoch != self._epoch:
                        return None
                    if self._turn[split_idx] != seq:
                        self._cv.wait(_POLL_S)
                        continue
                    q = self._queues[split_idx]
                    if q:
                        b, m = q.popleft()
                        self._stats["blocks"][split_idx] += 1
                        self._turn[split_idx] += 1
                        self._cv.notify_all()
                        return [b, m]
                    if self._done:
                        self._turn[split_idx] += 1
                        self._cv.notify_all()
                        return None
                    if not self._pulling:
                        self._pulling = True
                        break
                    self._cv.wait(_POLL_S)
            item = None
            rows = None
            try:
                item = next(self._it)
                # the block's row count is fetched BEFORE taking the lock: routing under _cv never
                # blocks on an object fetch, so other consumers' get / start_epoch calls proceed
                rows = self._rows(item[1])
            except StopIteration:
                pass
            except Exception:
                with self._cv:
                    self._pulling = False
                    self._done = True
                    self._cv.notify_all()
                raise
            with self._cv:
                self._pulling = False
                if epoch == self._epoch:
                    if item is None:
                        self._finish()
                    else:
                        self._route(item, split_idx, rows)
                self._cv.notify_all()

    def _rows(self, meta_ref) -> int:
        from ..._private.worker import get

        return int(get(meta_ref)["num_rows"])

    def _route(self, item, requester: int, rows: int):
        b, m = item
        if not self._equal:
            dest = requester
            if self._hints is not None:
                node = _block_node(b)
                if node is not None and self._hints[requester] != node:
                    for j, hint in enumerate(self._hints):
                        if hint == node and not self._queues[j]:
                            dest = j
                            break
            self._queues[dest].append((b, m))
            self._stats["rows"][dest] += rows
            return
        if rows == 0:
            return
        self._buffer.append((b, m, rows))
        self._buffer_rows += rows
        self._max_rows = max(self._max_rows, rows)
        keep = self._n * (self._max_rows + 1)
        # least-loaded dispatch keeps max(assigned) - min(assigned) <= max block rows; the hold-back
        # keeps enough rows to top every consumer up to the final target without overshooting it
        while self._buffer and self._buffer_rows - self._buffer[0][2] >= keep:
            hb, hm, hr = self._buffer.popleft()
            self._buffer_rows -= hr
            j = min(range(self._n), key=lambda i: (self._assigned[i], i))
            self._assigned[j] += hr
            self._queues[j].append((hb, hm))
            self._stats["rows"][j] += hr

    def _finish(self):
        self._done = True
        if not self._equal:
            return
        from . import execution as X

        target = (sum(self._assigned) + self._buffer_rows) // self._n
        cut = X._remote_fn(_slice_block, {"num_cpus": 0})
        for j in range(self._n):
            need = target - self._assigned[j]
            while need > 0 and self._buffer:
                b, m, r = self._buffer.popleft()
                self._buffer_rows -= r
                if r <= need:
                    self._queues[j].append((b, m))
                    need -= r
                    continue
                head = cut.remote(b, 0, need)
                tail = cut.remote(b, need, r)
                self._queues[j].append((head[0], head[1]))
                self._buffer.appendleft((tail[0], tail[1], r - need))
                self._buffer_rows += r - need
                need = 0
            self._stats["rows"][j] = target
        self._buffer.clear()
        self._buffer_rows = 0

    def stats(self):
        return dict(self._stats, epoch=self._epoch)

    def schema(self):
        return self._ds.schema()


def _slice_block(block, start, end):
    from ..block import BlockAccessor
    from .execution import _meta

    out = BlockAccessor(block).slice(start, end)
    return out, _meta(out)


def _block_node(ref) -> Optional[str]:
    try:
        from ..._private.worker import _core

        loc = getattr(_core(), "object_location", None)
        return loc(ref) if loc is not None else None
    except Exception:
        return None


class StreamSplitDataIterator(DataIterator):
    """Consumer ``split_idx`` of a streaming split: every iteration (``iter_batches`` /
    ``iter_rows`` / ``iter_torch_batches`` / ``materialize``) is one epoch of the shared execution."""

    def __init__(self, coord, split_idx: int, n: int, name: str = ""):
        super().__init__(None)
        self._coord = coord
        self._idx = split_idx
        self._n = n
        self._name = name

    def __reduce__(self):
        return StreamSplitDataIterator, (self._coord, self._idx, self._n, self._name)

    def schema(self):
        from ..._private.worker import get

        return get(self._coord.schema.remote())

    def __repr__(self):
        return f"StreamSplitDataIterator(split={self._idx}/{self._n}, dataset={self._name})"

    def _block_refs(self, prefetch: int):
        from ..._private.worker import get

        epoch = get(self._coord.start_epoch.remote(self._idx))
        seq = itertools.count()
        pending = collections.deque(self._coord.get.remote(epoch, self._idx, next(seq))
                                    for _ in range(max(1, prefetch + 1)))
        while pending:
            r = get(pending.popleft())
            if r is None:
                for p in pending:  # drain: the later calls answer None too
                    get(p)
                return
            pending.append(self._coord.get.remote(epoch, self._idx, next(seq)))
            yield r[0], r[1]

    def _blocks(self, prefetch: int):
        from ..._private.worker import get

        for b, _ in self._block_refs(prefetch):
            yield get(b)

    def materialize(self):
        from ..dataset import MaterializedDataset

        return MaterializedDataset(list(self._block_refs(1)))

    def stats(self):
        from ..._private.worker import get

        return str(get(self._coord.stats.remote()))


def streaming_split(ds, n: int, equal: bool = False, locality_hints=None) -> List[StreamSplitDataIterator]:
    from ... import remote

    if n <= 0:
        raise ValueError("streaming_split needs n >= 1")
    if locality_hints is not None and len(locality_hints) != n:
        raise ValueError(f"locality_hints must have {n} entries, got {len(locality_hints)}")
    hints = None
    if locality_hints is not None:
        hints = [h if isinstance(h, str) or h is None else getattr(h, "node_id", None) or str(h)
                 for h in locality_hints]
    cls = remote(num_cpus=0, max_concurrency=max(8, 4 * n + 4))(SplitCoordinator)
    coord = cls.remote(ds, n, equal, hints)  # returns at once: nothing executes until all n start epoch 0
    name = getattr(ds, "_name", None) or "dataset"
    return [StreamSplitDataIterator(coord, i, n, name) for i in range(n)]
