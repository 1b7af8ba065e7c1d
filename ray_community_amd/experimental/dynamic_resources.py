"""``ray.experimental.dynamic_resources`` import path."""
from . import set_resource

__all__ = ["set_resource"]
