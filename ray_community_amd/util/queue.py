"""Distributed FIFO queue backed by an async actor (reference: ``python/ray/util/queue.py``)."""
from __future__ import annotations

import asyncio
import queue as _q
from typing import Any, List, Optional


class Empty(_q.Empty):
    pass


class Full(_q.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize):
        self.maxsize = maxsize
        self.queue = asyncio.Queue(self.maxsize)

    def qsize(self):
        return self.queue.qsize()

    def empty(self):
        return self.queue.empty()

    def full(self):
        return self.queue.full()

    async def put(self, item, timeout=None):
        try:
            await asyncio.wait_for(self.queue.put(item), timeout)
        except asyncio.TimeoutError:
            raise Full

    async def put_batch(self, items, timeout=None):
        for item in items:
            try:
                await asyncio.wait_for(self.queue.put(item), timeout)
            except asyncio.TimeoutError:
                raise Full

    async def get(self, timeout=None):
        try:
            return await asyncio.wait_for(self.queue.get(), timeout)
        except asyncio.TimeoutError:
            raise Empty

    def put_nowait(self, item):
        self.queue.put_nowait(item)

    def put_nowait_batch(self, items):
        if self.maxsize > 0 and len(items) + self.qsize() > self.maxsize:
            raise Full(f"Cannot add {len(items)} items to queue of size {self.qsize()} and maxsize {self.maxsize}.")
        for item in items:
            self.queue.put_nowait(item)

    def get_nowait(self):
        return self.queue.get_nowait()

    def get_nowait_batch(self, num_items):
        if num_items > self.qsize():
            raise Empty(f"Cannot get {num_items} items from queue of size {self.qsize()}.")
        return [self.queue.get_nowait() for _ in range(num_items)]


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: Optional[dict] = None):
        from ..actor import ActorClass

        self.maxsize = maxsize
        opts = dict(actor_options or {})
        opts.setdefault("num_cpus", 0)
        self.actor = ActorClass(_QueueActor, opts).remote(self.maxsize)

    def __len__(self):
        return self.size()

    def size(self):
        return self.qsize()

    def qsize(self):
        from .._private.worker import get

        return get(self.actor.qsize.remote())

    def empty(self):
        from .._private.worker import get

        return get(self.actor.empty.remote())

    def full(self):
        from .._private.worker import get

        return get(self.actor.full.remote())

    def put(self, item, block=True, timeout=None):
        from .._private.worker import get

        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        if not block:
            try:
                get(self.actor.put_nowait.remote(item))
            except asyncio.QueueFull:
                raise Full
            except Exception as e:
                if "QueueFull" in type(e).__name__ or isinstance(e, asyncio.QueueFull):
                    raise Full
                raise
        else:
            try:
                get(self.actor.put.remote(item, timeout))
            except Full:
                raise
            except Exception as e:
                if isinstance(getattr(e, "cause", None), _q.Full):
                    raise Full
                raise

    async def put_async(self, item, block=True, timeout=None):
        if not block:
            return await self.actor.put_nowait.remote(item)
        return await self.actor.put.remote(item, timeout)

    def get(self, block=True, timeout=None):
        from .._private.worker import get

        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        try:
            if not block:
                return get(self.actor.get_nowait.remote())
            return get(self.actor.get.remote(timeout))
        except Exception as e:
            if isinstance(e, (_q.Empty, asyncio.QueueEmpty)) or isinstance(getattr(e, "cause", None),
                                                                            (_q.Empty, asyncio.QueueEmpty)):
                raise Empty
            raise

    async def get_async(self, block=True, timeout=None):
        if not block:
            return await self.actor.get_nowait.remote()
        return await self.actor.get.remote(timeout)

    def put_nowait(self, item):
        return self.put(item, block=False)

    def put_nowait_batch(self, items):
        from .._private.worker import get

        if not isinstance(items, list):
            raise TypeError("Argument 'items' must be a list")
        try:
            get(self.actor.put_nowait_batch.remote(items))
        except Exception as e:
            if isinstance(getattr(e, "cause", None), _q.Full) or isinstance(e, _q.Full):
                raise Full(str(e))
            raise

    def get_nowait(self):
        return self.get(block=False)

    def get_nowait_batch(self, num_items):
        from .._private.worker import get

        if not isinstance(num_items, int):
            raise TypeError("Argument 'num_items' must be an int")
        if num_items < 0:
            raise ValueError("'num_items' must be nonnegative")
        try:
            return get(self.actor.get_nowait_batch.remote(num_items))
        except Exception as e:
            if isinstance(getattr(e, "cause", None), _q.Empty) or isinstance(e, _q.Empty):
                raise Empty(str(e))
            raise

    def shutdown(self, force=False, grace_period_s=5):
        from .._private.worker import kill

        if self.actor:
            kill(self.actor)
        self.actor = None
