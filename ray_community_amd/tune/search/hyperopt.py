"""``ray.tune.search.hyperopt`` import path: HyperOptSearch is the native TPE searcher (tpe.py);
hyperopt itself is not installed."""
from .tpe import HyperOptSearch

__all__ = ["HyperOptSearch"]
