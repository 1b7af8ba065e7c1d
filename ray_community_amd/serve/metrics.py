"""Serve metrics (reference: python/ray/serve/metrics.py): ``util.metrics`` Counter / Gauge /
Histogram that inside a replica carry the ``deployment``, ``replica`` and ``application`` tags
by default, so user metrics line up with the built-in Serve ones on the dashboard's /metrics."""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from ..util import metrics as _m

_SERVE_TAGS = ("deployment", "replica", "application")


def _replica_tags() -> Dict[str, str]:
    try:
        from .api import get_replica_context

        ctx = get_replica_context()
    except Exception:  # noqa: BLE001 -- outside a replica: no default tags
        return {}
    return {"deployment": str(getattr(ctx, "deployment", "")), "replica": str(getattr(ctx, "replica_tag", "")),
            "application": str(getattr(ctx, "app_name", ""))}


def _with_serve_tags(cls):
    class _Serve(cls):
        def __init__(self, name: str, description: str = "", tag_keys: Optional[Tuple[str, ...]] = None, **kw):
            keys = tuple(tag_keys or ())
            for k in keys:
                if k in _SERVE_TAGS:
                    raise ValueError(f"'{k}' is reserved for Serve's default tags")
            super().__init__(name, description, tag_keys=keys + _SERVE_TAGS, **kw)
            tags = _replica_tags()
            if tags:
                self.set_default_tags(tags)

    _Serve.__name__ = _Serve.__qualname__ = cls.__name__
    return _Serve


Counter = _with_serve_tags(_m.Counter)
Gauge = _with_serve_tags(_m.Gauge)
Histogram = _with_serve_tags(_m.Histogram)

__all__ = ["Counter", "Gauge", "Histogram"]
