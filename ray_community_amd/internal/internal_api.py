"""Internal API (reference ``python/ray/internal/internal_api.py``): ``free`` (drop objects from
the object store ahead of their last reference) and ``memory_summary`` (the ``ray memory``
report as a string)."""
from __future__ import annotations

from typing import Optional


def free(object_refs, local_only: bool = False) -> None:
    from .._private.worker import free as _free

    _free(object_refs, local_only=local_only)


def memory_summary(address: Optional[str] = None, group_by: str = "NODE_ADDRESS", sort_by: str = "OBJECT_SIZE",
                   units: str = "B", line_wrap: bool = True, stats_only: bool = False, num_entries=None) -> str:
    """Object-store usage of the session: per-object rows (id, size, state, owner, call site) from
    the state API plus the store totals; ``stats_only`` keeps the totals."""
    from ..util.state import list_objects

    scale = {"B": 1, "KB": 1 << 10, "MB": 1 << 20, "GB": 1 << 30}.get(units, 1)
    objs = list_objects(limit=100000)
    total = sum(int(o.get("object_size") or 0) for o in objs)
    lines = ["======== Object references status ========",
             f"Objects: {len(objs)}  total size: {total / scale:.1f} {units}"]
    if not stats_only:
        key = {"OBJECT_SIZE": lambda o: -int(o.get("object_size") or 0),
               "REFERENCE_TYPE": lambda o: str(o.get("reference_type"))}.get(sort_by, lambda o: 0)
        rows = sorted(objs, key=key)
        if num_entries is not None:
            rows = rows[: int(num_entries)]
        lines.append(f"{'object id':44s} {'size':>12s} {'state':>10s} {'type':>14s}")
        for o in rows:
            lines.append(f"{str(o.get('object_id'))[:44]:44s} {int(o.get('object_size') or 0) / scale:12.1f} "
                         f"{str(o.get('state', '')):>10s} {str(o.get('reference_type', '')):>14s}")
    return "\n".join(lines)
