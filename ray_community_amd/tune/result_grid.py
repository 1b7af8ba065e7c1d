"""``ray.tune.result_grid`` import path."""
from .tuner import ResultGrid

__all__ = ["ResultGrid"]
