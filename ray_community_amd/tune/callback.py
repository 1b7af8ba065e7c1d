"""``ray.tune.callback`` import path."""
from . import Callback

__all__ = ["Callback"]
