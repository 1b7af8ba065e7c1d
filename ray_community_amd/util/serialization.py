"""Custom serializers (reference: ``python/ray/util/serialization.py``)."""
from .._private.serialization import deregister_serializer, register_serializer  # noqa: F401

__all__ = ["register_serializer", "deregister_serializer"]
