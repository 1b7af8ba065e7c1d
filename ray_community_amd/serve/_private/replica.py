"""Serve replica actor (reference: ``python/ray/serve/_private/replica.py``).

An async actor wrapping one instance of the user's deployment class (or function). Requests
arrive as actor calls; sync user methods run on a thread pool so the event loop keeps
accepting (and ``@serve.batch`` can coalesce) concurrent requests up to ``max_ongoing_requests``.
"""
from __future__ import annotations

import asyncio
import inspect
import os
import time
import traceback
from typing import Any, Dict, Optional

_REPLICA_CTX = {}


async def _aiter(res, executor=None):
    """Iterate a sync or async generator (a plain value yields once)."""
    if inspect.isasyncgen(res):
        async for x in res:
            yield x
    elif inspect.isgenerator(res):
        loop = asyncio.get_running_loop()
        done = object()
        while True:  # pull sync generator items on the user-code thread: the event loop keeps serving
            x = await loop.run_in_executor(executor, next, res, done)
            if x is done:
                break
            yield x
    else:
        yield res


class ReplicaContext:
    def __init__(self, app_name, deployment, replica_tag, servable_object=None):
        self.app_name = app_name
        self.deployment = deployment
        self.replica_tag = replica_tag
        self.replica_id = replica_tag
        self.servable_object = servable_object


class _JsonFormatter:
    """``LoggingConfig(encoding="JSON")``: one JSON object per record (reference
    ``serve/_private/logging_utils.py`` ServeJSONFormatter fields)."""

    def __init__(self, deployment, replica, app):
        import logging

        self._base = logging.Formatter()
        self.fields = {"deployment": deployment, "replica": replica, "application": app}

    def format(self, record):
        import json

        out = {"levelname": record.levelname, "asctime": self._base.formatTime(record), **self.fields,
               "message": record.getMessage()}
        for k in ("request_id", "route", "method", "status", "latency_ms"):
            if hasattr(record, k):
                out[k] = getattr(record, k)
        if record.exc_info:
            out["exc_text"] = self._base.formatException(record.exc_info)
        return json.dumps(out)


def configure_replica_logging(logging_config: Optional[Dict], app_name: str, deployment: str, tag: str):
    """Apply a deployment's ``LoggingConfig`` to the ``ray.serve`` logger of this replica process:
    level, TEXT/JSON encoding, a per-replica log file under ``logs_dir`` (default: the session's
    ``logs/serve``). Returns (logger, log file path)."""
    import logging

    lc = dict(logging_config or {})
    level = lc.get("log_level", "INFO")
    if isinstance(level, str):
        level = logging.getLevelName(level.upper())
        if not isinstance(level, int):
            raise ValueError(f"invalid log_level {lc.get('log_level')!r}")
    logs_dir = lc.get("logs_dir")
    if not logs_dir:
        from ..._private.worker import _core

        try:
            sess = _core().session_dir
        except Exception:
            sess = ""
        logs_dir = os.path.join(sess or "/tmp/rca_serve", "logs", "serve")
    os.makedirs(logs_dir, exist_ok=True)
    safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in tag)
    path = os.path.join(logs_dir, f"replica_{safe}_{os.getpid()}.log")
    logger = logging.getLogger("ray.serve")
    logger.setLevel(level)
    for h in [h for h in logger.handlers if getattr(h, "_rca_serve", False)]:
        logger.removeHandler(h)
        h.close()
    h = logging.FileHandler(path)
    h._rca_serve = True
    if str(lc.get("encoding", "TEXT")).upper() == "JSON":
        h.setFormatter(_JsonFormatter(deployment, tag, app_name))
    else:
        h.setFormatter(logging.Formatter(f"%(levelname)s %(asctime)s {deployment} {tag} -- %(message)s"))
    logger.addHandler(h)
    return logger, path


class ServeReplica:
    def __init__(self, app_name: str, deployment_name: str, replica_tag: str, body_blob: bytes, init_args, init_kwargs,
                 user_config=None, is_function: bool = False, logging_config: Optional[Dict] = None,
                 max_ongoing_requests: Optional[int] = None):
        from ..._private import serialization as ser
        from ..handle import _resolve_handle_args

        self.app_name = app_name
        self.deployment_name = deployment_name
        self.tag = replica_tag
        self.logging_config = dict(logging_config or {})
        self.logger, self.log_path = configure_replica_logging(logging_config, app_name, deployment_name, replica_tag)
        self.access_log = bool(self.logging_config.get("enable_access_log", True))
        body = ser.loads_function(body_blob)
        init_args, init_kwargs = _resolve_handle_args(init_args, init_kwargs)
        self.is_function = is_function
        _REPLICA_CTX["ctx"] = ReplicaContext(app_name, deployment_name, replica_tag)
        # ONE user-code thread (reference: replica.py ``_user_code_event_loop_thread``): the
        # constructor and every sync method run on it. Besides matching the reference's
        # semantics this keeps per-thread GPU library state warm: MIOpen / hipBLASLt handles are
        # per host thread, so a model warmed up in __init__ on thread A and served from a pool
        # thread B would pay kernel loading again (seconds per new thread for a ResNet-50).
        import concurrent.futures

        self._user_exec = concurrent.futures.ThreadPoolExecutor(max_workers=1, thread_name_prefix="serve-user")
        if is_function:
            self.obj = body
        else:
            self.obj = self._user_exec.submit(lambda: body(*init_args, **init_kwargs)).result()
            if inspect.isawaitable(self.obj):
                raise TypeError("constructor must not be async")
        _REPLICA_CTX["ctx"].servable_object = self.obj
        self.ongoing = 0
        self.total = 0
        self.started = time.time()
        # hard cap on user requests running at once (the actor's max_concurrency leaves headroom
        # for control calls): routers in other processes can over-commit on stale queue lengths,
        # so the excess waits here instead of running (reference: replica-side max_ongoing_requests)
        self.max_ongoing = int(max_ongoing_requests) if max_ongoing_requests else None
        if os.environ.get("RCA_SERVE_REPLICA_CAP", "1") == "0":  # A/B switch: router-side limits only
            self.max_ongoing = None
        self._slots = None
        self.peak_running = 0
        self._running = 0
        if user_config is not None:
            self._user_exec.submit(self._reconfigure_sync, user_config).result()

    def _slot(self):
        """Async context manager holding one of the replica's ``max_ongoing_requests`` slots."""
        import contextlib

        if self.max_ongoing is None:
            return contextlib.nullcontext()
        if self._slots is None:
            self._slots = asyncio.Semaphore(self.max_ongoing)
        replica = self

        class _Held:
            async def __aenter__(self):
                await replica._slots.acquire()
                replica._running += 1
                replica.peak_running = max(replica.peak_running, replica._running)

            async def __aexit__(self, *exc):
                replica._running -= 1
                replica._slots.release()
                return False

        return _Held()

    def _reconfigure_sync(self, user_config):
        fn = getattr(self.obj, "reconfigure", None)
        if fn is None:
            raise ValueError("user_config specified but deployment has no reconfigure() method")
        r = fn(user_config)
        if inspect.isawaitable(r):
            asyncio.get_event_loop().run_until_complete(r) if not asyncio.get_event_loop().is_running() else None

    async def reconfigure(self, user_config):
        fn = getattr(self.obj, "reconfigure", None)
        if fn is not None:
            r = fn(user_config)
            if inspect.isawaitable(r):
                await r
        return True

    async def _invoke_user(self, method_name, args, kwargs):
        """Call the user's method: coroutines awaited, sync code on the thread pool (the event
        loop keeps serving), generators returned unconsumed."""
        fn = self.obj if self.is_function else getattr(self.obj, method_name or "__call__")
        if inspect.iscoroutinefunction(fn) or inspect.iscoroutinefunction(getattr(fn, "__call__", None)):
            return await fn(*args, **kwargs)
        if inspect.isasyncgenfunction(fn):
            return fn(*args, **kwargs)
        loop = asyncio.get_running_loop()
        import contextvars

        ctx = contextvars.copy_context()
        res = await loop.run_in_executor(self._user_exec, lambda: ctx.run(fn, *args, **kwargs))
        if inspect.isawaitable(res):
            res = await res
        return res

    async def _call_user(self, method_name, args, kwargs, model_id=None):
        from .. import multiplex

        tok = multiplex._set_model_id(model_id)
        try:
            res = await self._invoke_user(method_name, args, kwargs)
            if inspect.isasyncgen(res):
                return [x async for x in res]
            if inspect.isgenerator(res):
                res = list(res)
            return res
        finally:
            multiplex._reset_model_id(tok)

    def _access(self, route, status, t0):
        """One access-log line per request (``LoggingConfig.enable_access_log``)."""
        if self.access_log:
            ms = 1000.0 * (time.time() - t0)
            self.logger.info(f"{route} {status} {ms:.1f}ms",
                             extra={"route": route, "status": status, "latency_ms": round(ms, 3)})

    def _grpc_kwargs(self, method_name, kwargs, meta):
        """A gRPC request's context goes to user methods that declare ``grpc_context``."""
        ctx = meta.get("grpc_context")
        if ctx is None:
            return kwargs
        from ..grpc_util import _wants_context

        fn = self.obj if self.is_function else getattr(self.obj, method_name or "__call__")
        return dict(kwargs, grpc_context=ctx) if _wants_context(fn) else kwargs

    async def handle_request(self, method_name, args, kwargs, meta=None):
        from ..handle import _resolve_handle_args

        meta = meta or {}
        self.ongoing += 1
        self.total += 1
        t0, status = time.time(), "OK"
        try:
            args, kwargs = _resolve_handle_args(args, kwargs)
            from ..._private.core_worker import ObjectRef

            # chained DeploymentResponses arrive as ObjectRefs: resolve them here, not in the caller
            args = tuple([(await a) if isinstance(a, ObjectRef) else a for a in args])
            kwargs = {k: ((await v) if isinstance(v, ObjectRef) else v) for k, v in kwargs.items()}
            kwargs = self._grpc_kwargs(method_name, kwargs, meta)
            async with self._slot():
                out = await self._call_user(method_name, args, kwargs, meta.get("multiplexed_model_id"))
            if meta.get("grpc_context") is not None:  # the (possibly modified) context rides back
                from ..grpc_util import _GrpcReply

                return _GrpcReply(out, kwargs.get("grpc_context", meta["grpc_context"]))
            return out
        except BaseException:
            status = "ERROR"
            raise
        finally:
            self.ongoing -= 1
            self._access(f"CALL {method_name or '__call__'}", status, t0)

    async def handle_request_stream(self, method_name, args, kwargs, meta=None):
        """Generator counterpart of ``handle_request`` for ``handle.options(stream=True)``:
        items of a (sync or async) generator method are streamed back one by one."""
        from ..handle import _resolve_handle_args
        from .. import multiplex

        meta = meta or {}
        self.ongoing += 1
        self.total += 1
        tok = multiplex._set_model_id(meta.get("multiplexed_model_id"))
        try:
            args, kwargs = _resolve_handle_args(args, kwargs)
            kwargs = self._grpc_kwargs(method_name, kwargs, meta)
            async with self._slot():
                res = await self._invoke_user(method_name, args, kwargs)
                async for x in _aiter(res, self._user_exec):
                    yield x
            if meta.get("grpc_context") is not None:  # last item: the context the stream left
                from ..grpc_util import _GrpcReply

                yield _GrpcReply(None, kwargs.get("grpc_context", meta["grpc_context"]))
        finally:
            multiplex._reset_model_id(tok)
            self.ongoing -= 1

    async def handle_http_stream(self, req: Dict):
        """Streaming HTTP: yields ("start", status, headers) then ("body", chunk) messages as the
        deployment produces them (ASGI apps, ``StreamingResponse``, generator ``__call__``)."""
        self.ongoing += 1
        self.total += 1
        try:
            from .http_util import stream_asgi_or_call

            async with self._slot():
                async for msg in stream_asgi_or_call(self, req):
                    yield msg
        finally:
            self.ongoing -= 1

    async def handle_http(self, req: Dict):
        """req: {method, path, query_string, headers, body, root_path}. Returns (status, headers, body)."""
        self.ongoing += 1
        self.total += 1
        t0, status = time.time(), 500
        try:
            from .http_util import run_asgi_or_call

            async with self._slot():
                out = await run_asgi_or_call(self, req)
            status = out[0] if isinstance(out, tuple) and out else 200
            return out
        finally:
            self.ongoing -= 1
            self._access(f"{req.get('method', 'GET')} {req.get('path', '/')}", status, t0)

    async def get_num_ongoing(self):
        return self.ongoing

    async def location(self):
        """Node and physical GPU ids of this replica (router locality: a request carrying a device
        tensor goes to a replica on the same GPU when one has room, saving an xGMI copy)."""
        from ..._private.worker import get_runtime_context
        from ..handle import physical_gpu_ids

        ctx = get_runtime_context()
        gpus = [int(g) for g in (ctx.get_accelerator_ids().get("GPU") or [])]
        return {"node_id": ctx.get_node_id(), "gpus": physical_gpu_ids(range(len(gpus))) if gpus else []}

    async def check_health(self):
        fn = getattr(self.obj, "check_health", None)
        if fn is not None:
            r = fn()
            if inspect.isawaitable(r):
                await r
        return True

    async def stats(self):
        return {"ongoing": self.ongoing, "total": self.total, "pid": os.getpid(), "tag": self.tag,
                "log_path": self.log_path}

    async def prepare_for_shutdown(self, wait_loop_s: float = 2.0, timeout_s: float = 20.0):
        """Graceful shutdown (reference replica.py perform_graceful_shutdown): the controller has
        already removed this replica from routing; sleep one wait-loop period so callers' routers
        see that, then poll until the ongoing requests drain (or ``timeout_s``), then run the
        user's destructor."""
        deadline = time.time() + max(0.0, timeout_s)
        await asyncio.sleep(max(0.0, min(wait_loop_s, timeout_s)))
        while self.ongoing > 0 and time.time() < deadline:
            await asyncio.sleep(min(max(wait_loop_s, 0.01), max(0.0, deadline - time.time())) or 0.01)
        d = getattr(self.obj, "__del__", None)
        if d is not None:
            try:
                r = d()
                if inspect.isawaitable(r):
                    await r
            except Exception:  # noqa  (a failing destructor must not block the shutdown)
                pass
        return self.ongoing
