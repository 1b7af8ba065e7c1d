"""Torch train-loop helpers (reference: ``python/ray/train/torch/train_loop_utils.py``)."""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import torch


def get_device() -> torch.device:
    idx = os.environ.get("RCA_TRAIN_DEVICE_INDEX")
    if torch.cuda.is_available():
        if idx is not None:
            return torch.device("cuda", int(idx))
        lr = os.environ.get("LOCAL_RANK")
        if lr is not None and int(lr) < torch.cuda.device_count():
            return torch.device("cuda", int(lr))
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def get_devices():
    return [get_device()]


def _world():
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def prepare_model(model: torch.nn.Module, move_to_device: bool = True, parallel_strategy: Optional[str] = "ddp",
                  parallel_strategy_kwargs: Optional[Dict[str, Any]] = None, wrap_ddp: Optional[bool] = None):
    """Move to the worker's device and wrap for data parallelism.

    ``parallel_strategy``: ``"ddp"`` (default) = the framework's bucketed RCCL DDP with flat
    gradient buckets (``ray_community_amd.parallel.DistributedDataParallel``); ``"torch_ddp"`` =
    ``torch.nn.parallel.DistributedDataParallel``; ``"fsdp"`` = torch FSDP; ``"zero3"`` = the
    framework's ZeRO-3 (``parallel.FullyShardedDataParallel``: per-block RCCL all-gather /
    reduce-scatter over flat shards; step it with ``parallel.FullyShardedAdamW`` and call
    ``finish_gradient_sync()`` after backward); ``None`` = no wrap.
    """
    kw = dict(parallel_strategy_kwargs or {})
    if wrap_ddp is False:
        parallel_strategy = None
    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    if _world() <= 1 or parallel_strategy is None:
        return model
    if parallel_strategy == "ddp":
        from ...parallel import DistributedDataParallel

        return DistributedDataParallel(model, bucket_cap_mb=kw.pop("bucket_cap_mb", 256.0),
                                       average_in_optimizer=False, auto_finalize=True)
    if parallel_strategy == "torch_ddp":
        from torch.nn.parallel import DistributedDataParallel as TDDP

        if dev.type == "cuda":
            kw.setdefault("device_ids", [dev.index])
        return TDDP(model, **kw)
    if parallel_strategy == "zero3":
        from ...parallel import FullyShardedDataParallel

        return FullyShardedDataParallel(model, **kw)
    if parallel_strategy == "fsdp":
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP

        return FSDP(model, device_id=dev if dev.type == "cuda" else None, **kw)
    raise ValueError(f"unknown parallel_strategy {parallel_strategy}")


class _DeviceLoader:
    def __init__(self, loader, device, auto_transfer=True):
        self._loader = loader
        self.device = device
        self._auto = auto_transfer
        self.dataset = getattr(loader, "dataset", None)
        self.sampler = getattr(loader, "sampler", None)
        self.batch_size = getattr(loader, "batch_size", None)

    def _move(self, x):
        if isinstance(x, torch.Tensor):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (list, tuple)):
            return type(x)(self._move(v) for v in x)
        if isinstance(x, dict):
            return {k: self._move(v) for k, v in x.items()}
        return x

    def __len__(self):
        return len(self._loader)

    def __iter__(self):
        for b in self._loader:
            yield self._move(b) if self._auto else b


def prepare_data_loader(data_loader, add_dist_sampler: bool = True, move_to_device: bool = True,
                        auto_transfer: bool = True):
    from torch.utils.data import DataLoader, DistributedSampler, IterableDataset, RandomSampler

    world = _world()
    if add_dist_sampler and world > 1 and not isinstance(data_loader.dataset, IterableDataset):
        import torch.distributed as dist

        shuffle = isinstance(data_loader.sampler, RandomSampler)
        sampler = DistributedSampler(data_loader.dataset, num_replicas=world, rank=dist.get_rank(), shuffle=shuffle)
        data_loader = DataLoader(data_loader.dataset, batch_size=data_loader.batch_size, sampler=sampler,
                                 num_workers=data_loader.num_workers, collate_fn=data_loader.collate_fn,
                                 pin_memory=data_loader.pin_memory, drop_last=data_loader.drop_last)
    if move_to_device:
        return _DeviceLoader(data_loader, get_device(), auto_transfer)
    return data_loader


def prepare_optimizer(optimizer):
    return optimizer


def backward(tensor):
    tensor.backward()


def enable_reproducibility(seed: int = 0):
    torch.manual_seed(seed)
    random.seed(seed)
    try:
        import numpy as np

        np.random.seed(seed)
    except ImportError:
        pass
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.benchmark = False


def accelerate(amp: bool = False):
    os.environ["RCA_TRAIN_AMP"] = "1" if amp else "0"


class TorchWorkerProfiler:  # pragma: no cover - kept for API parity
    def __init__(self, *a, **k):
        pass
