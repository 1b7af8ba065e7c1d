"""Data/model parallel building blocks over RCCL (xGMI) — MI355X-first replacements for the
reference's reliance on torch DDP/FSDP (``python/ray/train/torch/train_loop_utils.py``)."""
from .flat import FlatParameters
from .ddp import DistributedDataParallel
from .optim import FlatAdamW, FlatSGD
from .fsdp import ShardedAdamW, ShardedDataParallel
from .fully_sharded import FullyShardedAdamW, FullyShardedDataParallel, estimate_memory_gb

__all__ = ["FlatParameters", "DistributedDataParallel", "FlatAdamW", "FlatSGD", "ShardedDataParallel", "ShardedAdamW",
           "FullyShardedDataParallel", "FullyShardedAdamW", "estimate_memory_gb"]
