"""``ray.experimental.locations`` import path."""
from . import get_object_locations

__all__ = ["get_object_locations"]
