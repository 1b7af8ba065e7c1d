"""DataIterator (reference: ``python/ray/data/iterator.py``, ``_internal/block_batching``).

Blocks are prefetched ``prefetch_batches`` ahead (their producing tasks keep running while the
consumer works), re-batched to exactly ``batch_size`` rows, optionally locally shuffled, and — for
``iter_torch_batches`` — copied host->device with non-blocking transfers from pinned staging.
"""
from __future__ import annotations

import collections
from typing import Any, Callable, Dict, Iterator, Optional

import numpy as np

from .block import BlockAccessor, concat_blocks


class _IterableFromIterator:
    """What ``iter_batches`` / ``iter_torch_batches`` return: iterable any number of times (each
    ``iter()`` runs a fresh pass -- an epoch, for a training loop or a framework's data loader
    that re-iterates), and still an iterator itself (``next()`` draws from one lazily started pass)."""

    def __init__(self, make):
        self._make = make
        self._it = None

    def __iter__(self):
        return self._make()

    def __next__(self):
        if self._it is None:
            self._it = self._make()
        return next(self._it)


class DataIterator:
    def __init__(self, ds):
        self._ds = ds

    def _blocks(self, prefetch: int) -> Iterator:
        from .._private.worker import get, wait

        q = collections.deque()
        it = self._ds._iter_refs()
        done = False
        while True:
            while not done and len(q) < max(1, prefetch + 1):
                try:
                    q.append(next(it)[0])
                except StopIteration:
                    done = True
            if not q:
                return
            yield get(q.popleft())

    def iter_batches(self, **kw) -> Iterator:
        return _IterableFromIterator(lambda: self._iter_batches(**kw))

    def iter_torch_batches(self, **kw) -> Iterator:
        return _IterableFromIterator(lambda: self._iter_torch_batches(**kw))

    def _iter_batches(self, *, prefetch_batches: int = 1, batch_size: Optional[int] = 256,
                      batch_format: Optional[str] = "default", drop_last: bool = False,
                      local_shuffle_buffer_size: Optional[int] = None, local_shuffle_seed: Optional[int] = None,
                      _collate_fn=None) -> Iterator:
        rng = np.random.default_rng(local_shuffle_seed)
        buf = []
        buf_rows = 0
        min_rows = max(batch_size or 0, local_shuffle_buffer_size or 0)
        for blk in self._blocks(prefetch_batches):
            n = BlockAccessor(blk).num_rows()
            if n == 0:
                continue
            if batch_size is None:
                yield BlockAccessor(blk).to_batch(batch_format)
                continue
            buf.append(blk)
            buf_rows += n
            while buf_rows >= min_rows and buf_rows >= batch_size:
                merged = concat_blocks(buf)
                acc = BlockAccessor(merged)
                if local_shuffle_buffer_size:
                    merged = acc.take(rng.permutation(acc.num_rows()))
                    acc = BlockAccessor(merged)
                yield acc.slice(0, batch_size) if batch_format is None else BlockAccessor(
                    acc.slice(0, batch_size)).to_batch(batch_format)
                rest = acc.slice(batch_size, acc.num_rows())
                buf = [rest]
                buf_rows = acc.num_rows() - batch_size
        if buf_rows > 0 and not drop_last:
            merged = concat_blocks(buf)
            acc = BlockAccessor(merged)
            if local_shuffle_buffer_size:
                merged = acc.take(rng.permutation(acc.num_rows()))
                acc = BlockAccessor(merged)
            while acc.num_rows() > 0:
                k = min(batch_size, acc.num_rows())
                yield BlockAccessor(acc.slice(0, k)).to_batch(batch_format)
                merged = acc.slice(k, acc.num_rows())
                acc = BlockAccessor(merged)

    def iter_rows(self, *, prefetch_batches: int = 1) -> Iterator[Dict[str, Any]]:
        for blk in self._blocks(prefetch_batches):
            yield from BlockAccessor(blk).iter_rows()

    def _iter_torch_batches(self, *, prefetch_batches: int = 1, batch_size: Optional[int] = 256,
                            dtypes=None, device: str = "auto", collate_fn: Optional[Callable] = None,
                            drop_last: bool = False, local_shuffle_buffer_size=None, local_shuffle_seed=None,
                            pin_memory: bool = True) -> Iterator:
        import torch

        if device == "auto":
            from ..train.torch.train_loop_utils import get_device

            dev = get_device() if torch.cuda.is_available() else torch.device("cpu")
        else:
            dev = torch.device(device) if device is not None else torch.device("cpu")
        for b in self._iter_batches(prefetch_batches=prefetch_batches, batch_size=batch_size, batch_format="numpy",
                                   drop_last=drop_last, local_shuffle_buffer_size=local_shuffle_buffer_size,
                                   local_shuffle_seed=local_shuffle_seed):
            if collate_fn is not None:
                yield collate_fn(b)
                continue
            out = {}
            for k, v in b.items():
                if v.dtype == object:
                    out[k] = v
                    continue
                t = torch.as_tensor(np.ascontiguousarray(v))
                if dtypes is not None:
                    dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                    if dt is not None:
                        t = t.to(dt)
                if dev.type == "cuda":
                    if pin_memory:
                        t = t.pin_memory()
                    t = t.to(dev, non_blocking=True)
                out[k] = t
            yield out

    def to_tf(self, *a, **k):  # pragma: no cover
        raise ImportError("DataIterator.to_tf needs TensorFlow, which is not installed in this MI355X image")

    def iter_tf_batches(self, *a, **k):  # pragma: no cover
        raise ImportError("DataIterator.iter_tf_batches needs TensorFlow, which is not installed in this MI355X image")

    def schema(self):
        """Schema of the underlying dataset (reference ``DataIterator.schema``)."""
        ds = self._ds
        return ds.schema() if hasattr(ds, "schema") else None

    def to_torch(self, *, label_column=None, feature_columns=None, batch_size: int = 1, **kw):
        """A ``torch.utils.data.IterableDataset`` over this iterator's batches: ``(features,
        label)`` tensors with ``label_column``, else the batch dicts (reference ``to_torch``)."""
        import torch

        it = self

        class _It(torch.utils.data.IterableDataset):
            def __iter__(_s):
                for b in it.iter_torch_batches(batch_size=batch_size):
                    if label_column:
                        y = b.pop(label_column)
                        cols = feature_columns or list(b)
                        yield torch.stack([b[c].float() for c in cols], dim=1), y
                    else:
                        yield b

        return _It()

    def materialize(self):
        return self._ds.materialize()

    def stats(self):
        return self._ds.stats()
