"""Native data-parallel histogram GBDT (engine of ``train.xgboost`` / ``train.lightgbm``)."""
from .core import Booster, DMatrix, Tree, TrainingCallback, normalize_params, train

__all__ = ["Booster", "DMatrix", "Tree", "TrainingCallback", "normalize_params", "train"]
