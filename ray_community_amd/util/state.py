"""State API (reference: ``python/ray/util/state/api.py``): list/get/summarize cluster entities."""
from __future__ import annotations

from collections import Counter
from typing import Any, Dict, List, Optional, Tuple


def _call(method, *args):
    from .._private.worker import _core

    return _core().client.call(method, *args)


def _filter(rows, filters):
    if not filters:
        return rows
    out = []
    for r in rows:
        ok = True
        for key, op, val in filters:
            v = r.get(key)
            if op in ("=", "==") and str(v) != str(val):
                ok = False
            elif op == "!=" and str(v) == str(val):
                ok = False
        if ok:
            out.append(r)
    return out


def list_actors(filters: Optional[List[Tuple[str, str, Any]]] = None, limit: int = 10000, detail=False, **kw):
    return _filter(_call("list_actors"), filters)[:limit]


def list_tasks(filters=None, limit: int = 10000, detail=False, **kw):
    _flush_own_task_records()
    return _filter(_call("list_tasks", limit), filters)[:limit]


def _flush_own_task_records():
    """Leased tasks are reported to the head by their submitter in batches: this process's
    pending records go first, so its own finished tasks are listed."""
    from .._private.core_worker import global_core

    try:
        c = global_core()
    except Exception:  # noqa
        return
    if c is not None and c.task_records:
        recs, c.task_records = c.task_records, []
        c.client.call("direct_task_records", recs)


def list_objects(filters=None, limit: int = 10000, detail=False, **kw):
    return _filter(_call("list_objects"), filters)[:limit]


def list_nodes(filters=None, limit: int = 10000, detail=False, **kw):
    rows = [{"node_id": n["NodeID"], "state": "ALIVE" if n["Alive"] else "DEAD", "is_head_node": n["IsHead"],
             "resources_total": n["Resources"], "labels": n.get("Labels", {})} for n in _call("nodes")]
    return _filter(rows, filters)[:limit]


def list_workers(filters=None, limit: int = 10000, detail=False, **kw):
    return _filter(_call("list_workers"), filters)[:limit]


def list_placement_groups(filters=None, limit: int = 10000, detail=False, **kw):
    return _filter(list(_call("pg_table", None).values()), filters)[:limit]


def get_actor(id: str):
    for a in list_actors():
        if a["actor_id"] == id:
            return a
    return None


def get_task(id: str):
    for t in list_tasks():
        if t["task_id"] == id:
            return t
    return None


def summarize_tasks(**kw) -> Dict[str, Any]:
    by = {}
    for t in list_tasks():
        d = by.setdefault(t["func_or_class_name"], {"func_or_class_name": t["func_or_class_name"],
                                                     "type": t["type"], "state_counts": Counter()})
        d["state_counts"][t["state"]] += 1
    for d in by.values():
        d["state_counts"] = dict(d["state_counts"])
    return {"cluster": {"summary": by, "total_tasks": sum(sum(d["state_counts"].values()) for d in by.values())}}


def summarize_actors(**kw):
    by = {}
    for a in list_actors():
        d = by.setdefault(a["class_name"], {"class_name": a["class_name"], "state_counts": Counter()})
        d["state_counts"][a["state"]] += 1
    for d in by.values():
        d["state_counts"] = dict(d["state_counts"])
    return {"cluster": {"summary": by, "total_actors": sum(sum(d["state_counts"].values()) for d in by.values())}}


def summarize_objects(**kw):
    objs = list_objects()
    return {"cluster": {"total_objects": len(objs), "total_size_mb": sum(o["object_size"] or 0 for o in objs) / 2**20}}


def object_store_stats():
    return _call("store_stats")
