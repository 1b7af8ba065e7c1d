"""``ray.tune.tune_config`` import path."""
from .tuner import TuneConfig

__all__ = ["TuneConfig"]
