"""``request_resources`` (reference: ``python/ray/autoscaler/sdk/sdk.py``): command the
autoscaler to keep capacity for the given shapes regardless of current load; each call replaces
the previous request (``request_resources()`` clears it)."""
from __future__ import annotations

import json
from typing import Dict, List, Optional


def request_resources(num_cpus: Optional[int] = None, bundles: Optional[List[Dict[str, float]]] = None) -> None:
    from .._private.core_worker import global_core

    shapes: List[Dict[str, float]] = []
    if num_cpus:
        shapes += [{"CPU": 1.0}] * int(num_cpus)
    for b in bundles or []:
        shapes.append({k: float(v) for k, v in b.items() if v})
    global_core().client.call("kv_put", "__autoscaler_resource_request__", json.dumps(shapes).encode(), True,
                              "autoscaler")
