"""``ray.tune.experiment`` (reference ``python/ray/tune/experiment/``): the Trial and Experiment
classes."""
from ..registry import Experiment
from ..tuner import Trial

__all__ = ["Experiment", "Trial"]
