"""Experimental APIs (reference: ``python/ray/experimental/__init__.py``)."""
from typing import Any, Dict, List


def get_object_locations(obj_refs: List, timeout_ms: int = -1) -> Dict[Any, Dict[str, Any]]:
    """Map each ref to ``{"node_ids": [...], "object_size": bytes}``; refs whose location is
    unknown (still pending, or freed) are left out (reference: ``experimental/locations.py``)."""
    from .._private import worker as w

    if not w.is_initialized():
        raise RuntimeError("Ray hasn't been initialized.")
    refs = list(obj_refs)
    locs = w._core().client.call("object_locations", [r._id for r in refs])
    return {r: locs[r._id] for r in refs if r._id in locs}


def set_resource(resource_name: str, capacity: float, node_id=None):
    """Dynamic custom resources were removed from the reference (it raises); same here."""
    raise DeprecationWarning("Dynamic custom resources are deprecated. Consider using placement groups instead "
                             "(docs.ray.io/en/master/placement-group.html). You can also specify resources at Ray "
                             "start time with the 'resources' field in the cluster autoscaler.")


def load_package(config_path: str):
    """A code package with its own runtime environment (``experimental/packaging``)."""
    from .packaging import load_package as _load

    return _load(config_path)


__all__ = ["get_object_locations", "set_resource", "load_package"]
