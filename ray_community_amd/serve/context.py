"""``ray.serve.context`` import path: the replica context of the running request."""
from ._private.replica import ReplicaContext
from .api import get_replica_context

__all__ = ["ReplicaContext", "get_replica_context"]
