"""``ray.train.context`` import path (reference: python/ray/train/context.py)."""
from ._internal.session import TrainContext


def get_context() -> TrainContext:
    from . import get_context as _g

    return _g()


__all__ = ["TrainContext", "get_context"]
