"""``multiprocessing.Pool`` on actors (reference: ``python/ray/util/multiprocessing/pool.py``)."""
from __future__ import annotations

import itertools
import threading
from multiprocessing import JoinableQueue, TimeoutError  # noqa: A004  (same names as the stdlib module)
from typing import Any, Callable, Iterable, List, Optional


class _PoolWorker:
    def __init__(self, initializer=None, initargs=()):
        if initializer:
            initializer(*initargs)

    def run_batch(self, fn, batch, star=False):
        if star:
            return [fn(*args) for args in batch]
        return [fn(x) for x in batch]


class AsyncResult:
    def __init__(self, refs, single=False, callback=None, error_callback=None, chunked=True):
        self._refs = refs
        self._single = single
        self._callback = callback
        self._error_callback = error_callback
        self._result = None
        self._done = False
        self._lock = threading.Lock()
        self._fired = False
        if callback is not None or error_callback is not None:
            # like multiprocessing's result-handler thread: callbacks fire on completion, not on get()
            self._pending = len(refs)
            for r in refs:
                r.future().add_done_callback(self._on_done)

    def _on_done(self, _fut):
        with self._lock:
            self._pending -= 1
            if self._pending > 0:
                return
        try:
            self.get(timeout=0)
        except Exception:
            pass

    def get(self, timeout=None):
        from .._private.worker import get

        if not self._done:
            try:
                out = get(self._refs, timeout=timeout)
                flat = list(itertools.chain.from_iterable(out))
                self._result = flat[0] if self._single else flat
                self._done = True
                self._fire(self._callback, self._result)
            except Exception as e:
                from ..exceptions import GetTimeoutError

                if isinstance(e, GetTimeoutError):
                    raise TimeoutError(str(e)) from e  # multiprocessing's contract
                self._fire(self._error_callback, e)
                raise
        return self._result

    def _fire(self, cb, arg):
        with self._lock:
            if self._fired or cb is None:
                return
            self._fired = True
        cb(arg)

    def wait(self, timeout=None):
        from .._private.worker import wait

        wait(self._refs, num_returns=len(self._refs), timeout=timeout)

    def ready(self):
        from .._private.worker import wait

        r, _ = wait(self._refs, num_returns=len(self._refs), timeout=0)
        return len(r) == len(self._refs)

    def successful(self):
        try:
            self.get(timeout=0)
            return True
        except Exception:
            return False


class Pool:
    def __init__(self, processes: Optional[int] = None, initializer=None, initargs=(), maxtasksperchild=None,
                 context=None, ray_remote_args: Optional[dict] = None, ray_address=None):
        from .._private import worker as w
        from ..actor import ActorClass

        if not w.is_initialized():
            w.init(address=ray_address)
        if processes is None:
            processes = int(w.cluster_resources().get("CPU", 1))
        if processes < 1:
            raise ValueError("Processes in the pool must be >0.")
        opts = dict(ray_remote_args or {})
        opts.setdefault("num_cpus", 1)
        cls = ActorClass(_PoolWorker, opts)
        self._actors = [cls.remote(initializer, initargs) for _ in range(processes)]
        self._processes = processes
        self._closed = False
        self._rr = 0

    def _chunks(self, iterable, chunksize):
        items = list(iterable)
        if chunksize is None:
            chunksize = max(1, len(items) // (self._processes * 4) + (1 if len(items) % (self._processes * 4) else 0))
        return [items[i: i + chunksize] for i in range(0, len(items), chunksize)]

    def _submit(self, fn, batches, star=False):
        if self._closed:
            raise ValueError("Pool not running")
        refs = []
        for b in batches:
            a = self._actors[self._rr % len(self._actors)]
            self._rr += 1
            refs.append(a.run_batch.remote(fn, b, star))
        return refs

    def apply(self, func, args=(), kwds=None):
        return self.apply_async(func, args, kwds).get()

    def apply_async(self, func, args=(), kwds=None, callback=None, error_callback=None):
        kwds = kwds or {}
        f = (lambda *a: func(*a, **kwds)) if kwds else func
        refs = self._submit(f, [[tuple(args)]], star=True)
        return AsyncResult(refs, single=True, callback=callback, error_callback=error_callback)

    def map(self, func, iterable, chunksize=None):
        return self.map_async(func, iterable, chunksize).get()

    def map_async(self, func, iterable, chunksize=None, callback=None, error_callback=None):
        return AsyncResult(self._submit(func, self._chunks(iterable, chunksize)), callback=callback,
                           error_callback=error_callback)

    def starmap(self, func, iterable, chunksize=None):
        return self.starmap_async(func, iterable, chunksize).get()

    def starmap_async(self, func, iterable, chunksize=None, callback=None, error_callback=None):
        return AsyncResult(self._submit(func, self._chunks([tuple(x) for x in iterable], chunksize), star=True),
                           callback=callback, error_callback=error_callback)

    def imap(self, func, iterable, chunksize=1):
        from .._private.worker import get

        for r in self._submit(func, self._chunks(iterable, chunksize)):
            yield from get(r)

    def imap_unordered(self, func, iterable, chunksize=1):
        from .._private.worker import get, wait

        pending = self._submit(func, self._chunks(iterable, chunksize))
        while pending:
            ready, pending = wait(pending, num_returns=1)
            yield from get(ready[0])

    def close(self):
        self._closed = True

    def terminate(self):
        from .._private.worker import kill

        self._closed = True
        for a in self._actors:
            try:
                kill(a)
            except Exception:
                pass
        self._actors = []

    def join(self):
        if not self._closed:
            raise ValueError("Pool is still running")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.terminate()
