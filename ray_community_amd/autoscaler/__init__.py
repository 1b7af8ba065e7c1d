"""Autoscaler (reference: ``python/ray/autoscaler/`` -- ``sdk.request_resources``,
``_private/autoscaler.py`` StandardAutoscaler, ``_private/resource_demand_scheduler.py``,
``node_provider.py``; config keys ``available_node_types``, ``min_workers``/``max_workers``,
``idle_timeout_minutes``, ``upscaling_speed``).

On one MI355X box the nodes the autoscaler manages are *virtual* nodes of the session (resource
pools with their own worker pools, as ``cluster_utils`` uses) -- e.g. carve the 8 GPUs into
``gpu_worker`` nodes of 1 GPU only while work needs them. The provider interface is the same
shape as the reference's so other providers can be plugged in.

Each :meth:`StandardAutoscaler.update`:
  1. reads the head's load: resource shapes of queued tasks/actors, pending placement-group
     bundles, per-node totals/availability/busy workers, and the standing
     ``request_resources`` request;
  2. bin-packs queued demand onto free capacity (nodes being launched count with their full
     shape), then the standing request onto TOTAL capacity; each shape that does not fit starts
     the first node type that can hold it (``max_workers`` per type and overall, at most
     ``upscaling_speed`` x current workers + 1 launches per update), and ``min_workers`` are
     kept;
  3. terminates autoscaler-launched nodes that stayed idle (nothing running, every resource
     free) for ``idle_timeout_minutes`` unless needed for ``min_workers`` or the request.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional

from .sdk import request_resources  # noqa: F401

_REQUEST_KEY = "__autoscaler_resource_request__"
TYPE_LABEL = "ray.io/node-type"


class NodeProvider:
    """Interface (reference: ``python/ray/autoscaler/node_provider.py``)."""

    def create_node(self, node_type: str, resources: Dict[str, float], labels: Dict[str, str]) -> str:
        raise NotImplementedError

    def terminate_node(self, node_id: str) -> None:
        raise NotImplementedError

    def non_terminated_nodes(self) -> Dict[str, str]:
        """{node_id: node_type} of the nodes this provider launched."""
        raise NotImplementedError


class VirtualNodeProvider(NodeProvider):
    """Virtual nodes of the session this process hosts (the head runs in-process)."""

    def __init__(self):
        self._nodes: Dict[str, str] = {}

    def _head(self):
        from .._private import worker

        head = worker._state.get("head")
        if head is None:
            raise RuntimeError("VirtualNodeProvider needs the process that hosts the session's head")
        return head

    def create_node(self, node_type, resources, labels):
        nid = self._head().add_node(dict(resources), dict(labels))
        self._nodes[nid] = node_type
        return nid

    def terminate_node(self, node_id):
        self._head().remove_node(node_id)
        self._nodes.pop(node_id, None)

    def non_terminated_nodes(self):
        alive = {n["node_id"] for n in _client().call("node_load")}
        for nid in [n for n in self._nodes if n not in alive]:
            self._nodes.pop(nid, None)
        return dict(self._nodes)


def _client():
    from .._private.core_worker import global_core

    return global_core().client


def _fits(demand: Dict[str, float], avail: Dict[str, float]) -> bool:
    return all(avail.get(k, 0.0) + 1e-9 >= v for k, v in demand.items())


def _take(demand, avail):
    for k, v in demand.items():
        avail[k] = avail.get(k, 0.0) - v


def _binpack(demands: List[Dict[str, float]], bins: List[Dict[str, float]]) -> List[Dict[str, float]]:
    """First-fit-decreasing of ``demands`` into ``bins`` (mutated); returns what did not fit."""
    unmet = []
    for d in sorted(demands, key=lambda d: -sum(d.values())):
        for b in bins:
            if _fits(d, b):
                _take(d, b)
                break
        else:
            unmet.append(d)
    return unmet


class StandardAutoscaler:
    def __init__(self, config: Dict, provider: Optional[NodeProvider] = None):
        """``config``: ``{"available_node_types": {name: {"resources": {...}, "min_workers": 0,
        "max_workers": N, "labels": {...}}}, "max_workers": M, "idle_timeout_minutes": T,
        "upscaling_speed": U}``."""
        self.types = config.get("available_node_types") or {}
        if not self.types:
            raise ValueError("autoscaler config needs available_node_types")
        self.max_workers = int(config.get("max_workers", sum(int(t.get("max_workers", 0)) for t in self.types.values())))
        self.idle_timeout_s = float(config.get("idle_timeout_minutes", 5.0)) * 60.0
        self.upscaling_speed = float(config.get("upscaling_speed", 1.0))
        self.provider = provider or VirtualNodeProvider()
        self._idle_since: Dict[str, float] = {}
        self._thread = None
        self._stop = threading.Event()
        self.events: List[str] = []

    # ------------------------------------------------------------------ decisions
    def _counts(self, nodes: Dict[str, str]) -> Dict[str, int]:
        c = {t: 0 for t in self.types}
        for t in nodes.values():
            c[t] = c.get(t, 0) + 1
        return c

    def _pick_type(self, demand, counts, total) -> Optional[str]:
        if total >= self.max_workers:
            return None
        for name, t in self.types.items():
            if counts.get(name, 0) < int(t.get("max_workers", 0)) and _fits(demand, dict(t.get("resources", {}))):
                return name
        return None

    def update(self) -> Dict:
        cl = _client()
        load = cl.call("node_load")
        dem = cl.call("resource_demands")
        req = _standing_request(cl)
        nodes = self.provider.non_terminated_nodes()
        counts = self._counts(nodes)
        total = len(nodes)
        launched, terminated = [], []
        budget = max(1, int(self.upscaling_speed * max(1, total)))

        def launch(name):
            nonlocal total
            t = self.types[name]
            nid = self.provider.create_node(name, dict(t.get("resources", {})), {TYPE_LABEL: name, **t.get("labels", {})})
            counts[name] = counts.get(name, 0) + 1
            total += 1
            launched.append((name, nid))
            self.events.append(f"launched {name} {nid[:8]}")
            return nid

        # queued demand on free capacity (placement-group bundles: STRICT_PACK as one shape)
        demands = list(dem["tasks"])
        for pg in dem["placement_groups"]:
            if pg["strategy"] == "STRICT_PACK":
                merged: Dict[str, float] = {}
                for b in pg["bundles"]:
                    for k, v in b.items():
                        merged[k] = merged.get(k, 0.0) + v
                demands.append(merged)
            else:
                demands.extend(pg["bundles"])
        free = [dict(n["available"]) for n in load]
        unmet = _binpack(demands, free)
        # standing request_resources bundles against TOTAL capacity
        tot = [dict(n["total"]) for n in load]
        unmet_req = _binpack(list(req), tot)
        new_free: List[Dict[str, float]] = []  # leftovers of nodes started in this update
        for d in unmet + unmet_req:
            if not _binpack([d], new_free):
                continue  # shares a node started for an earlier shape
            if len(launched) >= budget:
                break
            name = self._pick_type(d, counts, total)
            if name is None:
                continue  # no node type can hold it (or every type is at max_workers)
            launch(name)
            rest = dict(self.types[name].get("resources", {}))
            _take(d, rest)
            new_free.append(rest)
        for name, t in self.types.items():
            while counts.get(name, 0) < int(t.get("min_workers", 0)) and total < self.max_workers:
                launch(name)
        # scale down idle autoscaler nodes
        now = time.time()
        by_id = {n["node_id"]: n for n in load}
        needed_for_request = bool(req) and not unmet_req
        for nid, name in list(nodes.items()):
            n = by_id.get(nid)
            if n is None:
                continue
            idle = n["busy_workers"] == 0 and all(abs(n["available"].get(k, 0.0) - v) < 1e-6 for k, v in n["total"].items())
            if not idle:
                self._idle_since.pop(nid, None)
                continue
            t0 = self._idle_since.setdefault(nid, now)
            if now - t0 < self.idle_timeout_s:
                continue
            if counts.get(name, 0) <= int(self.types.get(name, {}).get("min_workers", 0)):
                continue
            if needed_for_request and not _request_fits_without(req, load, nid):
                continue
            self.provider.terminate_node(nid)
            counts[name] -= 1
            self._idle_since.pop(nid, None)
            terminated.append((name, nid))
            self.events.append(f"terminated idle {name} {nid[:8]}")
            load = [x for x in load if x["node_id"] != nid]
        return {"launched": launched, "terminated": terminated, "pending_demands": len(demands),
                "unmet": len(unmet) + len(unmet_req), "workers": dict(counts)}

    # ------------------------------------------------------------------ monitor loop
    @property
    def all_node_types(self):
        return set(self.types)

    def summary(self) -> Dict:
        """Active nodes per type and the configured bounds (reference ``StandardAutoscaler.summary``)."""
        nodes = self.provider.non_terminated_nodes()
        counts = self._counts(nodes)
        return {"active_nodes": counts, "num_nodes": len(nodes), "max_workers": self.max_workers,
                "node_types": {n: {"min_workers": int(t.get("min_workers", 0)),
                                   "max_workers": int(t.get("max_workers", 0))} for n, t in self.types.items()}}

    def info_string(self) -> str:
        s = self.summary()
        lines = ["======== Autoscaler status ========", "Node types (active / min / max):"]
        for n, b in sorted(s["node_types"].items()):
            lines.append(f"  {n}: {s['active_nodes'].get(n, 0)} / {b['min_workers']} / {b['max_workers']}")
        lines.append(f"Total nodes: {s['num_nodes']} (max workers {s['max_workers']})")
        return "\n".join(lines)

    def reset(self, errors_fatal: bool = False) -> None:
        """Forget idle timers (a config reload in the reference)."""
        self._idle_since = {}

    def start(self, interval_s: float = 1.0) -> "StandardAutoscaler":
        def loop():
            while not self._stop.wait(interval_s):
                try:
                    self.update()
                except Exception as e:  # noqa - keep monitoring
                    self.events.append(f"update failed: {e!r}")

        self._thread = threading.Thread(target=loop, name="rca-autoscaler", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)


def _standing_request(cl) -> List[Dict[str, float]]:
    import json

    raw = cl.call("kv_get", _REQUEST_KEY, "autoscaler")
    if not raw:
        return []
    return [dict(b) for b in json.loads(raw)]


def _request_fits_without(req, load, drop_id) -> bool:
    return not _binpack(list(req), [dict(n["total"]) for n in load if n["node_id"] != drop_id])
