"""Core utilities (reference: ``python/ray/util``)."""
from .placement_group import (PlacementGroup, get_current_placement_group, get_placement_group, placement_group,
                              placement_group_table, remove_placement_group)
from .scheduling_strategies import (NodeAffinitySchedulingStrategy, NodeLabelSchedulingStrategy,
                                    PlacementGroupSchedulingStrategy)


def get_node_ip_address():
    return "127.0.0.1"


def __getattr__(name):
    import importlib

    if name in ("collective", "queue", "actor_pool", "multiprocessing", "metrics", "state", "iter", "serialization",
                "annotations", "timer", "tracing"):
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
           "Queue", "inspect_serializability"]
