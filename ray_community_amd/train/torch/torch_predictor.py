"""``ray.train.torch.torch_predictor`` import path."""
from .torch_checkpoint import TorchPredictor

__all__ = ["TorchPredictor"]
