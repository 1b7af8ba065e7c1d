"""``ray.train.base_trainer`` import path (reference: python/ray/train/base_trainer.py)."""
from ._internal.backend_executor import TrainingFailedError
from .data_parallel_trainer import BaseTrainer

GenDataset = object  # Dataset or a callable returning one

__all__ = ["BaseTrainer", "TrainingFailedError", "GenDataset"]
