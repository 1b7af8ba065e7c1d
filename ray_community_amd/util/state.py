"""State API (reference: ``python/ray/util/state/api.py``): list/get/summarize cluster entities."""
from __future__ import annotations

from collections import Counter
import contextlib
import os
import threading
from typing import Any, Dict, Iterator, List, Optional, Tuple

_LOCAL = threading.local()


@contextlib.contextmanager
def warnings_on_slow_request(*, address: str, endpoint: str, timeout: float, explain: bool):
    """Log a warning at timeout/8, /4 and /2 while a state request is still waiting (only when
    ``explain``); reference util/state/api.py."""
    if not explain:
        yield
        return
    import logging
    import time

    log = logging.getLogger("ray_community_amd.util.state")
    t0 = time.monotonic()
    timers = [threading.Timer(timeout * f, lambda f=f: log.warning(
        f"({round(time.monotonic() - t0, 2)} / {timeout} seconds) waiting for the response from {address}{endpoint}"))
              for f in (1 / 8, 1 / 4, 1 / 2)]
    for t in timers:
        t.daemon = True
        t.start()
    try:
        yield
    finally:
        for t in timers:
            t.cancel()


def _call(method, *args):
    c = getattr(_LOCAL, "client", None)  # the dashboard answering /api/v0 with its own head link
    if c is not None:
        return c.call(method, *args)
    from .._private.worker import _core

    return _core().client.call(method, *args)


@contextlib.contextmanager
def _using_client(client):
    prev = getattr(_LOCAL, "client", None)
    _LOCAL.client = client
    try:
        yield
    finally:
        _LOCAL.client = prev


_RESOURCES = ("actors", "tasks", "objects", "nodes", "workers", "placement_groups", "jobs", "runtime_envs",
              "cluster_events")


def _http_list(address: str, resource: str, filters, limit: int, detail: bool):
    """List through a dashboard's ``/api/v0/<resource>`` (reference state-API HTTP protocol)."""
    import requests

    params = [("limit", str(limit)), ("detail", str(bool(detail)))]
    for k, op, v in filters or []:
        params += [("filter_keys", k), ("filter_predicates", op), ("filter_values", str(v))]
    base = address if address.startswith("http") else "http://" + address
    r = requests.get(f"{base.rstrip('/')}/api/v0/{resource}", params=params, timeout=30)
    r.raise_for_status()
    body = r.json()
    if not body.get("result", False):
        raise RuntimeError(body.get("msg") or f"state API request for {resource} failed")
    return body["data"]["result"]["result"]


def _remote(kw) -> Optional[str]:
    a = kw.get("address")
    return a if isinstance(a, str) and (a.startswith("http") or ":" in a and not a.startswith("ray://")) else None


_PREDICATES = ("=", "==", "!=")


def _match(v, val) -> bool:
    if isinstance(v, bool) or isinstance(val, bool):
        return str(v).lower() == str(val).lower()
    return str(v) == str(val)


def _filter(rows, filters):
    """AND of ``(key, predicate, value)`` filters; predicates ``=`` / ``!=`` as in the reference
    (``util/state/common.py`` ``ListApiOptions``), values compared as strings (booleans
    case-insensitively, so ``("is_detached", "=", "true")`` works from the CLI too)."""
    if not filters:
        return rows
    for f in filters:
        if len(f) != 3 or f[1] not in _PREDICATES:
            raise ValueError(f"Unsupported filter {f!r}: use (key, '=' | '!=', value)")
    out = []
    for r in rows:
        ok = True
        for key, op, val in filters:
            eq = _match(r.get(key), val)
            if (op == "!=") == eq:
                ok = False
                break
        if ok:
            out.append(r)
    return out


def list_actors(filters: Optional[List[Tuple[str, str, Any]]] = None, limit: int = 10000, detail=False, **kw):
    if _remote(kw):
        return _http_list(_remote(kw), "actors", filters, limit, detail)
    return _filter(_call("list_actors"), filters)[:limit]


def list_tasks(filters=None, limit: int = 10000, detail=False, **kw):
    if _remote(kw):
        return _http_list(_remote(kw), "tasks", filters, limit, detail)
    if getattr(_LOCAL, "client", None) is None:
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
    if _remote(kw):
        return _http_list(_remote(kw), "objects", filters, limit, detail)
    return _filter(_call("list_objects"), filters)[:limit]


def list_nodes(filters=None, limit: int = 10000, detail=False, **kw):
    if _remote(kw):
        return _http_list(_remote(kw), "nodes", filters, limit, detail)
    rows = [{"node_id": n["NodeID"], "state": "ALIVE" if n["Alive"] else "DEAD", "is_head_node": n["IsHead"],
             "resources_total": n["Resources"], "labels": n.get("Labels", {})} for n in _call("nodes")]
    return _filter(rows, filters)[:limit]


def list_workers(filters=None, limit: int = 10000, detail=False, **kw):
    if _remote(kw):
        return _http_list(_remote(kw), "workers", filters, limit, detail)
    return _filter(_call("list_workers"), filters)[:limit]


def list_placement_groups(filters=None, limit: int = 10000, detail=False, **kw):
    if _remote(kw):
        return _http_list(_remote(kw), "placement_groups", filters, limit, detail)
    return _filter(list(_call("pg_table", None).values()), filters)[:limit]


def list_jobs(filters=None, limit: int = 10000, detail=False, **kw):
    """The driver job of this session plus submitted jobs (job submission manager), reference
    ``list_jobs`` fields: ``job_id``/``submission_id``, ``type``, ``status``, ``entrypoint``."""
    if _remote(kw):
        return _http_list(_remote(kw), "jobs", filters, limit, detail)
    from .._private.worker import _core

    core = _core()
    rows = [{"job_id": core.job_id.hex() if isinstance(core.job_id, bytes) else str(core.job_id),
             "submission_id": None, "type": "DRIVER", "status": "RUNNING", "entrypoint": "",
             "driver_info": {"pid": os.getpid()}}]
    try:
        from ..job_submission import _job_manager
        from .._private.worker import get

        mgr = _job_manager(create=False)
        for d in get(mgr.list.remote(), timeout=10):
            st = d.get("status")
            rows.append({"job_id": d.get("submission_id"), "submission_id": d.get("submission_id"),
                         "type": "SUBMISSION", "status": getattr(st, "value", st),
                         "entrypoint": d.get("entrypoint"), "message": d.get("message"),
                         "start_time": d.get("start_time"), "end_time": d.get("end_time"),
                         "metadata": d.get("metadata")})
    except Exception:  # noqa  (no job has been submitted in this session)
        pass
    return _filter(rows, filters)[:limit]


def list_runtime_envs(filters=None, limit: int = 10000, detail=False, **kw):
    """Distinct runtime environments of the live workers (one row per env, with its worker count)."""
    if _remote(kw):
        return _http_list(_remote(kw), "runtime_envs", filters, limit, detail)
    rows = {}
    for w in _call("list_workers"):
        key = str(w.get("runtime_env") or {})
        r = rows.setdefault(key, {"runtime_env": w.get("runtime_env") or {}, "success": True, "ref_cnt": 0})
        r["ref_cnt"] += 1
    return _filter(list(rows.values()), filters)[:limit]


def list_cluster_events(filters=None, limit: int = 10000, detail=False, **kw):
    """Node / worker / OOM-kill events recorded by the head (reference: ``list_cluster_events``)."""
    if _remote(kw):
        return _http_list(_remote(kw), "cluster_events", filters, limit, detail)
    return _filter(_call("cluster_events"), filters)[:limit]


def list_logs(node_id: Optional[str] = None, glob_filter: Optional[str] = None, **kw) -> Dict[str, List[str]]:
    """``{node_id: [log file names]}`` (worker stdout/stderr files ``worker-<id>.out``)."""
    return _call("list_logs", node_id, glob_filter)


def get_log(filename: Optional[str] = None, actor_id: Optional[str] = None, task_id: Optional[str] = None,
            pid: Optional[int] = None, node_id: Optional[str] = None, tail: int = -1, follow: bool = False,
            interval: float = 0.5, worker_id: Optional[str] = None, **kw) -> Iterator[str]:
    """Yield the lines of one worker log, found by file name, actor id, task id, worker id or pid
    (reference: ``util/state/api.py`` ``get_log``). ``follow=True`` keeps yielding new lines."""
    import time

    if task_id is not None:
        _flush_own_task_records()  # leased tasks: the worker that ran it is in this process's records
    lines = _call("get_log", filename, actor_id, task_id, pid, worker_id, tail)
    yield from lines
    if not follow:
        return
    seen = len(_call("get_log", filename, actor_id, task_id, pid, worker_id, -1))
    while True:
        time.sleep(interval)
        try:
            cur = _call("get_log", filename, actor_id, task_id, pid, worker_id, -1)
        except Exception:  # noqa  (the worker is gone)
            return
        yield from cur[seen:]
        seen = len(cur)


def get_actor(id: str):
    for a in list_actors():
        if a["actor_id"] == id:
            return a
    return None


def get_task(id: str):
    """The latest attempt of a task (reference returns the attempt list's last entry)."""
    hit = None
    for t in list_tasks():
        if t["task_id"] == id:
            hit = t
    return hit


def get_node(id: str):
    return next((n for n in list_nodes() if n["node_id"] == id), None)


def get_worker(id: str):
    return next((w for w in list_workers() if w["worker_id"] == id), None)


def get_placement_group(id: str):
    return next((p for p in list_placement_groups() if p.get("placement_group_id") == id), None)


def get_job(id: str):
    return next((j for j in list_jobs() if id in (j["job_id"], j.get("submission_id"))), None)


def get_objects(id: str):
    return [o for o in list_objects() if o["object_id"] == id]


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


class StateApiClient:
    """Object form of the state API (reference ``util/state/api.py::StateApiClient``): ``list(resource)``,
    ``get(resource, id)``, ``summary(resource)`` over the module functions."""

    _LIST = {"actors": "list_actors", "tasks": "list_tasks", "objects": "list_objects", "nodes": "list_nodes",
             "workers": "list_workers", "placement_groups": "list_placement_groups", "jobs": "list_jobs",
             "runtime_envs": "list_runtime_envs", "cluster_events": "list_cluster_events"}
    _GET = {"actors": "get_actor", "tasks": "get_task", "nodes": "get_node", "workers": "get_worker",
            "placement_groups": "get_placement_group", "jobs": "get_job", "objects": "get_objects"}

    def __init__(self, address: Optional[str] = None, cookies=None, headers=None):
        self.address = address

    def list(self, resource, options=None, raise_on_missing_output: bool = True, _explain: bool = False):
        r = getattr(resource, "value", resource)
        filters = getattr(options, "filters", None) if options is not None else None
        limit = getattr(options, "limit", 10000) if options is not None else 10000
        return globals()[self._LIST[r]](filters=filters, limit=limit)

    def get(self, resource, id: str, options=None, _explain: bool = False):
        return globals()[self._GET[getattr(resource, "value", resource)]](id)

    def summary(self, resource, *, options=None, raise_on_missing_output: bool = True, _explain: bool = False):
        return globals()[f"summarize_{getattr(resource, 'value', resource)}"]()
