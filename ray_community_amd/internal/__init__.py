"""``ray.internal`` (reference ``python/ray/internal/__init__.py``): the internal API module."""
from . import internal_api
from .internal_api import free, memory_summary

__all__ = ["free", "memory_summary", "internal_api"]
