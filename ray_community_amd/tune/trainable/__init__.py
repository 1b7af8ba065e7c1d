"""``ray.tune.trainable`` import path (reference: python/ray/tune/trainable/): the class API
``Trainable``, function trainables (any ``f(config)`` that calls ``tune.report``), and
``with_parameters`` / ``with_resources``."""
from .. import with_parameters, with_resources
from ..tuner import Trainable

FunctionTrainable = Trainable  # function trainables run inside the same trial actor machinery


def wrap_function(train_func, *args, **kwargs):
    """Function trainables are used as they are (the controller runs them in a trial thread)."""
    return train_func


__all__ = ["Trainable", "FunctionTrainable", "with_parameters", "with_resources", "wrap_function"]
