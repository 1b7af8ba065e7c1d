"""``@serve.batch`` (reference: ``python/ray/serve/batching.py``): concurrent calls to an async
method are coalesced into one call on a list, up to ``max_batch_size`` or ``batch_wait_timeout_s``."""
from __future__ import annotations

import asyncio
import functools
import inspect
from typing import Any, Callable, List, Optional


class _BatchQueue:
    def __init__(self, fn, max_batch_size, timeout_s, owner):
        self.fn = fn
        self.max = max_batch_size
        self.timeout = timeout_s
        self.owner = owner
        self.q: asyncio.Queue = asyncio.Queue()
        self.task = asyncio.get_running_loop().create_task(self._loop())

    async def _loop(self):
        while True:
            first = await self.q.get()
            items = [first]
            deadline = asyncio.get_running_loop().time() + self.timeout
            while len(items) < self.max:
                rem = deadline - asyncio.get_running_loop().time()
                if rem <= 0:
                    break
                try:
                    items.append(await asyncio.wait_for(self.q.get(), rem))
                except asyncio.TimeoutError:
                    break
            args = [x[0] for x in items]
            futs = [x[1] for x in items]
            try:
                res = self.fn(self.owner, args) if self.owner is not None else self.fn(args)
                if inspect.isawaitable(res):
                    res = await res
                res = list(res)
                if len(res) != len(items):
                    raise ValueError(f"batched function returned {len(res)} results for a batch of {len(items)}")
                for f, r in zip(futs, res):
                    if not f.done():
                        f.set_result(r)
            except Exception as e:  # noqa
                for f in futs:
                    if not f.done():
                        f.set_exception(e)


def batch(_func=None, *, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.0):
    if max_batch_size < 1:
        raise ValueError("max_batch_size must be at least 1")

    def deco(fn):
        if not inspect.iscoroutinefunction(fn):
            raise TypeError("Functions decorated with @serve.batch must be 'async def'")
        params = list(inspect.signature(fn).parameters)
        is_method = bool(params) and params[0] == "self"
        attr = f"__rca_batch_queue_{fn.__name__}"

        if is_method:
            @functools.wraps(fn)
            async def wrapper(self, arg):
                q = self.__dict__.get(attr)
                if q is None:
                    q = _BatchQueue(fn, max_batch_size, batch_wait_timeout_s, self)
                    self.__dict__[attr] = q
                f = asyncio.get_running_loop().create_future()
                await q.q.put((arg, f))
                return await f
        else:
            holder = {}

            @functools.wraps(fn)
            async def wrapper(arg):
                q = holder.get("q")
                if q is None:
                    q = _BatchQueue(fn, max_batch_size, batch_wait_timeout_s, None)
                    holder["q"] = q
                f = asyncio.get_running_loop().create_future()
                await q.q.put((arg, f))
                return await f

        wrapper._rca_batch = (max_batch_size, batch_wait_timeout_s)
        return wrapper

    return deco(_func) if _func is not None else deco
