"""``ray.train.session`` import path: the per-worker session functions."""
from . import get_checkpoint, get_context, get_dataset_shard, report  # noqa: F401

__all__ = ["report", "get_checkpoint", "get_context", "get_dataset_shard"]
