"""Application metrics (reference: ``python/ray/util/metrics.py``).

Counter / Gauge / Histogram with tag keys, recorded per process and exported in Prometheus text
format (``export_prometheus``) — the reference pipes them through the dashboard agent.
"""
from __future__ import annotations

import threading
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

_REGISTRY: Dict[str, "Metric"] = {}
_LOCK = threading.Lock()


class Metric:
    kind = "untyped"

    def __init__(self, name: str, description: str = "", tag_keys: Optional[Tuple[str, ...]] = None):
        _ensure_pusher()
        if not name:
            raise ValueError("Empty name is not allowed. Please provide a metric name.")
        if tag_keys is not None and not isinstance(tag_keys, tuple):
            raise TypeError(f"tag_keys should be a tuple type, got: {type(tag_keys)}")
        self._name = name
        self._description = description
        self._tag_keys = tuple(tag_keys or ())
        self._default_tags: Dict[str, str] = {}
        self._values: Dict[tuple, float] = defaultdict(float)
        with _LOCK:
            _REGISTRY[name] = self

    def set_default_tags(self, default_tags: Dict[str, str]):
        for k in default_tags:
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
        self._default_tags = dict(default_tags)
        return self

    def _key(self, tags):
        t = dict(self._default_tags)
        t.update(tags or {})
        for k in t:
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
        missing = [k for k in self._tag_keys if k not in t]
        if missing:
            raise ValueError(f"Missing value for tag key(s): {','.join(missing)}.")
        return tuple((k, str(t[k])) for k in self._tag_keys)

    @property
    def info(self):
        return {"name": self._name, "description": self._description, "tag_keys": self._tag_keys,
                "default_tags": self._default_tags}

    def _samples(self):
        return [(self._name, dict(k), v) for k, v in self._values.items()]


class Counter(Metric):
    kind = "counter"

    def inc(self, value: float = 1.0, tags: Optional[Dict[str, str]] = None):
        if value <= 0:
            raise ValueError(f"value must be >0, got {value}")
        self._values[self._key(tags)] += value


class Gauge(Metric):
    kind = "gauge"

    def set(self, value: float, tags: Optional[Dict[str, str]] = None):
        self._values[self._key(tags)] = float(value)


class Histogram(Metric):
    kind = "histogram"

    def __init__(self, name, description="", boundaries: Optional[List[float]] = None, tag_keys=None):
        if not boundaries:
            raise ValueError("boundaries must be a non-empty list")
        if any(b <= 0 for b in boundaries) or sorted(boundaries) != list(boundaries):
            raise ValueError("boundaries must be positive and increasing")
        super().__init__(name, description, tag_keys)
        self.boundaries = list(boundaries)
        self._buckets: Dict[tuple, List[int]] = {}
        self._sum: Dict[tuple, float] = defaultdict(float)
        self._count: Dict[tuple, int] = defaultdict(int)

    def observe(self, value: float, tags: Optional[Dict[str, str]] = None):
        k = self._key(tags)
        b = self._buckets.setdefault(k, [0] * (len(self.boundaries) + 1))
        i = 0
        while i < len(self.boundaries) and value > self.boundaries[i]:
            i += 1
        b[i] += 1
        self._sum[k] += value
        self._count[k] += 1

    def _samples(self):
        out = []
        for k, b in self._buckets.items():
            tags = dict(k)
            acc = 0
            for bound, n in zip(self.boundaries + [float("inf")], b):
                acc += n
                out.append((self._name + "_bucket", {**tags, "le": str(bound)}, acc))
            out.append((self._name + "_sum", tags, self._sum[k]))
            out.append((self._name + "_count", tags, self._count[k]))
        return out


def export_prometheus() -> str:
    lines = []
    with _LOCK:
        metrics = list(_REGISTRY.values())
    for m in metrics:
        lines.append(f"# HELP {m._name} {m._description}")
        lines.append(f"# TYPE {m._name} {m.kind}")
        for name, tags, v in m._samples():
            t = ",".join(f'{k}="{val}"' for k, val in tags.items())
            lines.append(f"{name}{{{t}}} {v}" if t else f"{name} {v}")
    return "\n".join(lines) + "\n"


# ------------------------------------------------------------------ push to the head
_PUSHER = {"thread": None}


def _ensure_pusher(period_s: float = 2.0):
    """Every process that records metrics pushes its exposition text to the head (which serves
    the cluster-wide ``/metrics`` of the dashboard)."""
    if _PUSHER["thread"] is not None:
        return
    import os

    def loop():
        import time

        src = f"{os.uname().nodename}:{os.getpid()}"
        while True:
            time.sleep(period_s)
            try:
                from .._private.worker import _core, is_initialized

                if is_initialized():
                    _core().client.call("metrics_push", src, export_prometheus())
            except Exception:
                pass

    _PUSHER["thread"] = threading.Thread(target=loop, daemon=True, name="rca-metrics-push")
    _PUSHER["thread"].start()
