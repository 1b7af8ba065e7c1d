"""Core utilities (reference: ``python/ray/util``)."""
from .placement_group import (PlacementGroup, get_current_placement_group, get_placement_group, placement_group,
                              placement_group_table, remove_placement_group)
from .scheduling_strategies import (NodeAffinitySchedulingStrategy, NodeLabelSchedulingStrategy,
                                    PlacementGroupSchedulingStrategy)


from .debug import disable_log_once_globally, enable_periodic_logging, log_once
from .._private.serialization import deregister_serializer, register_serializer


def get_node_ip_address():
    return "127.0.0.1"


def list_named_actors(all_namespaces: bool = False):
    """Names of the live named actors in this job's namespace (``{"name", "namespace"}`` dicts
    across every namespace with ``all_namespaces=True``), as ``ray.util.list_named_actors``."""
    from .._private import worker as w
    from .state import list_actors

    ns = w._state.get("namespace")
    out = []
    for a in list_actors():
        if not a.get("name") or a.get("state") == "DEAD":
            continue
        if all_namespaces:
            out.append({"name": a["name"], "namespace": a.get("namespace")})
        elif a.get("namespace") == ns:
            out.append(a["name"])
    return out


def connect(conn_str: str, **kw):
    """Ray Client: drive a remote session (``ray://host:port``) from this process."""
    from .._private import worker as w

    addr = conn_str if conn_str.startswith("ray://") else "ray://" + conn_str
    return w.init(address=addr, **kw)


def disconnect():
    from .._private import worker as w

    w.shutdown()


def __getattr__(name):
    import importlib

    if name in ("collective", "queue", "actor_pool", "multiprocessing", "metrics", "state", "iter", "serialization",
                "annotations", "timer", "tracing", "accelerators", "pdb", "debug", "client", "ray_debugpy"):
        return importlib.import_module("." + name, __name__)
    if name == "ActorPool":
        from .actor_pool import ActorPool

        return ActorPool
    if name == "Queue":
        from .queue import Queue

        return Queue
    if name == "inspect_serializability":
        from .check_serialize import inspect_serializability

        return inspect_serializability
    raise AttributeError(name)


__all__ = ["PlacementGroup", "placement_group", "placement_group_table", "remove_placement_group",
           "get_placement_group", "get_current_placement_group", "PlacementGroupSchedulingStrategy",
           "NodeAffinitySchedulingStrategy", "NodeLabelSchedulingStrategy", "get_node_ip_address", "ActorPool",
           "Queue", "inspect_serializability", "accelerators", "log_once", "disable_log_once_globally",
           "enable_periodic_logging", "pdb", "connect", "disconnect", "register_serializer", "deregister_serializer",
           "list_named_actors"]
