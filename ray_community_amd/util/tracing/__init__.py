"""Distributed tracing across tasks and actors (reference: ``python/ray/util/tracing/
tracing_helper.py``, which wraps every remote call in an OpenTelemetry span and propagates the
context inside the task spec).

OpenTelemetry is not installed in this image, so the span model is built in: a span is
``(trace_id, span_id, parent_id, name, start, end, attributes)``. When tracing is enabled
(``ray.init(_tracing_startup_hook=...)`` or :func:`enable_tracing`), every task / actor
submission carries the submitter's current span context; the executing worker opens a child span
``task::<name>`` (or ``actor_method::<Class.method>``) around the call and makes it current, so
nested submissions and user spans (:func:`start_span`) chain into the same trace. Finished spans
are shipped to the head with the task's completion message; :func:`get_spans` /
:func:`export_spans` read them back, and ``ray.timeline()`` shows them next to the task events.
``ray._private.profiling.profile`` records spans the same way whether or not tracing is on.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from typing import Dict, List, Optional

_local = threading.local()
_enabled = False
_buffer: List[dict] = []
_buf_lock = threading.Lock()


def _new_id(nbytes: int) -> str:
    return os.urandom(nbytes).hex()


def enable_tracing(enabled: bool = True) -> None:
    global _enabled
    _enabled = bool(enabled)


def is_tracing_enabled() -> bool:
    return _enabled or current_span_context() is not None


def current_span_context() -> Optional[tuple]:
    """(trace_id, span_id) of the span active on this thread, or None."""
    stack = getattr(_local, "stack", None)
    return stack[-1] if stack else None


def _push(ctx):
    if not hasattr(_local, "stack"):
        _local.stack = []
    _local.stack.append(ctx)


def _pop():
    _local.stack.pop()


def _record(span: dict) -> None:
    with _buf_lock:
        _buffer.append(span)
        overflow = len(_buffer) > 100000
        if overflow:
            del _buffer[: len(_buffer) - 100000]


def drain() -> List[dict]:
    """Spans finished in this process since the last drain (shipped to the head)."""
    with _buf_lock:
        out = list(_buffer)
        _buffer.clear()
    return out


@contextlib.contextmanager
def start_span(name: str, attributes: Optional[Dict] = None, parent: Optional[tuple] = None, kind: str = "internal"):
    """Open a span (child of ``parent`` or of the current span; a new trace otherwise) and make it
    current for the enclosed block."""
    par = parent if parent is not None else current_span_context()
    trace_id = par[0] if par else _new_id(16)
    ctx = (trace_id, _new_id(8))
    span = {"trace_id": trace_id, "span_id": ctx[1], "parent_id": par[1] if par else None, "name": name,
            "kind": kind, "start": time.time(), "end": None, "pid": os.getpid(),
            "thread": threading.get_ident(), "attributes": dict(attributes or {}), "status": "ok"}
    _push(ctx)
    try:
        yield span
    except BaseException as e:
        span["status"] = "error"
        span["attributes"]["exception"] = f"{type(e).__name__}: {e}"
        raise
    finally:
        _pop()
        span["end"] = time.time()
        _record(span)


def submission_context() -> Optional[tuple]:
    """Context to embed in a task spec at submission: the current span, or a fresh root when
    tracing is enabled but no span is active."""
    ctx = current_span_context()
    if ctx is not None:
        return ctx
    if _enabled:
        return (_new_id(16), None)
    return None


def _flush_to_head() -> None:
    spans = drain()
    if not spans:
        return
    from ..._private.worker import _core

    _core().client.call("add_spans", spans)


def get_spans(trace_id: Optional[str] = None) -> List[dict]:
    """All finished spans the cluster has collected (optionally one trace), sorted by start."""
    from ..._private.worker import _core

    _flush_to_head()
    spans = _core().client.call("spans")
    if trace_id is not None:
        spans = [s for s in spans if s["trace_id"] == trace_id]
    return sorted(spans, key=lambda s: s["start"])


def export_spans(path: str, trace_id: Optional[str] = None) -> int:
    """Write spans as JSON lines (one span per line); returns the count."""
    spans = get_spans(trace_id)
    with open(path, "w") as f:
        for s in spans:
            f.write(json.dumps(s) + "\n")
    return len(spans)


def setup_tracing(hook: Optional[str]) -> None:
    """``_tracing_startup_hook="module:function"``: call it (it may configure exporters) and turn
    tracing on."""
    if hook:
        if callable(hook):
            hook()
        else:
            import importlib

            mod, _, fn = str(hook).partition(":")
            if fn:
                getattr(importlib.import_module(mod), fn)()
    enable_tracing(True)


__all__ = ["enable_tracing", "is_tracing_enabled", "start_span", "current_span_context", "get_spans",
           "export_spans", "setup_tracing"]
