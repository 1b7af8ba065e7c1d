"""``ray.tune.search.optuna`` import path: OptunaSearch is the native TPE searcher (tpe.py);
optuna itself is not installed."""
from .tpe import OptunaSearch

__all__ = ["OptunaSearch"]
