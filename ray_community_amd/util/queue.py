"""Distributed FIFO queue (API of ``python/ray/util/queue.py``).

The queue lives in one async actor (``_QueueServer``): a ``collections.deque`` plus two
``asyncio.Condition`` s -- ``_not_empty`` (getters park on it) and ``_not_full`` (putters park on
it while a bounded queue is at capacity). Blocking calls with a timeout are implemented as a
bounded wait on the matching condition, so a parked call never holds the actor's event loop.
The server reports "would block" by returning a status tag instead of raising, and the client
turns it into ``queue.Empty`` / ``queue.Full``.
"""
from __future__ import annotations

import asyncio
import collections
import queue as _stdq
from typing import Any, List, Optional

_OK, _EMPTY, _FULL = "ok", "empty", "full"


class Empty(_stdq.Empty):
    pass


class Full(_stdq.Full):
    pass


class _QueueServer:
    def __init__(self, capacity: int):
        self._cap = capacity if capacity and capacity > 0 else 0
        self._items: collections.deque = collections.deque()
        self._lock = asyncio.Lock()
        self._not_empty = asyncio.Condition(self._lock)
        self._not_full = asyncio.Condition(self._lock)

    def _room(self, n: int = 1) -> bool:
        return self._cap == 0 or len(self._items) + n <= self._cap

    # introspection
    def qsize(self) -> int:
        return len(self._items)

    def empty(self) -> bool:
        return not self._items

    def full(self) -> bool:
        return self._cap > 0 and len(self._items) >= self._cap

    async def _wait_for(self, cond: asyncio.Condition, pred, timeout: Optional[float]) -> bool:
        try:
            await asyncio.wait_for(cond.wait_for(pred), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    # producers
    async def put(self, items: List[Any], block: bool, timeout: Optional[float]):
        async with self._lock:
            for x in items:
                if not self._room():
                    if not block or not await self._wait_for(self._not_full, self._room, timeout):
                        return _FULL
                self._items.append(x)
                self._not_empty.notify()
            return _OK

    async def put_all_or_nothing(self, items: List[Any]):
        async with self._lock:
            if not self._room(len(items)):
                return (_FULL, f"Cannot add {len(items)} items to queue of size {len(self._items)} and "
                               f"maxsize {self._cap}.")
            self._items.extend(items)
            self._not_empty.notify(len(items))
            return (_OK, None)

    # consumers
    async def get(self, block: bool, timeout: Optional[float]):
        async with self._lock:
            if not self._items:
                if not block or not await self._wait_for(self._not_empty, lambda: bool(self._items), timeout):
                    return (_EMPTY, None)
            x = self._items.popleft()
            self._not_full.notify()
            return (_OK, x)

    async def get_exactly(self, n: int):
        async with self._lock:
            if n > len(self._items):
                return (_EMPTY, f"Cannot get {n} items from queue of size {len(self._items)}.")
            out = [self._items.popleft() for _ in range(n)]
            self._not_full.notify(n)
            return (_OK, out)


class Queue:
    """``Queue(maxsize=0)``: a FIFO shared by every process holding this object."""

    def __init__(self, maxsize: int = 0, actor_options: Optional[dict] = None):
        from ..actor import ActorClass

        self.maxsize = maxsize
        opts = {"num_cpus": 0, **(actor_options or {})}
        self.actor = ActorClass(_QueueServer, opts).remote(maxsize)

    @staticmethod
    def _sync(ref):
        from .._private.worker import get

        return get(ref)

    @staticmethod
    def _check_timeout(timeout):
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")

    def __len__(self) -> int:
        return self.size()

    def size(self) -> int:
        return self.qsize()

    def qsize(self) -> int:
        return self._sync(self.actor.qsize.remote())

    def empty(self) -> bool:
        return self._sync(self.actor.empty.remote())

    def full(self) -> bool:
        return self._sync(self.actor.full.remote())

    # ------------------------------------------------------------------ put
    def put(self, item, block: bool = True, timeout: Optional[float] = None):
        self._check_timeout(timeout)
        if self._sync(self.actor.put.remote([item], block, timeout)) == _FULL:
            raise Full

    async def put_async(self, item, block: bool = True, timeout: Optional[float] = None):
        self._check_timeout(timeout)
        if await self.actor.put.remote([item], block, timeout) == _FULL:
            raise Full

    def put_nowait(self, item):
        return self.put(item, block=False)

    def put_nowait_batch(self, items: list):
        if not isinstance(items, list):
            raise TypeError("Argument 'items' must be a list")
        status, msg = self._sync(self.actor.put_all_or_nothing.remote(items))
        if status == _FULL:
            raise Full(msg)

    # ------------------------------------------------------------------ get
    def get(self, block: bool = True, timeout: Optional[float] = None):
        self._check_timeout(timeout)
        status, item = self._sync(self.actor.get.remote(block, timeout))
        if status == _EMPTY:
            raise Empty
        return item

    async def get_async(self, block: bool = True, timeout: Optional[float] = None):
        self._check_timeout(timeout)
        status, item = await self.actor.get.remote(block, timeout)
        if status == _EMPTY:
            raise Empty
        return item

    def get_nowait(self):
        return self.get(block=False)

    def get_nowait_batch(self, num_items: int):
        if not isinstance(num_items, int):
            raise TypeError("Argument 'num_items' must be an int")
        if num_items < 0:
            raise ValueError("'num_items' must be nonnegative")
        status, out = self._sync(self.actor.get_exactly.remote(num_items))
        if status == _EMPTY:
            raise Empty(out)
        return out

    def shutdown(self, force: bool = False, grace_period_s: int = 5):
        from .._private.worker import kill

        if self.actor is not None:
            kill(self.actor)
        self.actor = None
