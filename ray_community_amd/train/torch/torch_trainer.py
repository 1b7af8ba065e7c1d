"""TorchTrainer (reference: ``python/ray/train/torch/torch_trainer.py``)."""
from __future__ import annotations

import os
from datetime import timedelta
from typing import Any, Callable, Dict, Optional

from ..data_parallel_trainer import DataParallelTrainer
from .config import TorchConfig


class TorchTrainer(DataParallelTrainer):
    """Data-parallel PyTorch training: one actor per worker (``num_gpus=1`` each with
    ``use_gpu=True``), process group over RCCL (GPU) or gloo (CPU)."""

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[Dict] = None,
                 torch_config: Optional[TorchConfig] = None, scaling_config=None, run_config=None, datasets=None,
                 dataset_config=None, metadata=None, resume_from_checkpoint=None):
        super().__init__(train_loop_per_worker, train_loop_config=train_loop_config,
                         backend_config=torch_config or TorchConfig(), scaling_config=scaling_config,
                         run_config=run_config, datasets=datasets, dataset_config=dataset_config,
                         resume_from_checkpoint=resume_from_checkpoint, metadata=metadata)

    def _setup_external_backend(self):
        import torch
        import torch.distributed as dist

        if dist.is_initialized():
            return
        world = int(os.environ.get("WORLD_SIZE", "1"))
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        use_gpu = self.scaling_config.use_gpu and torch.cuda.is_available()
        kw = {}
        if use_gpu:
            torch.cuda.set_device(lr)
            os.environ["RCA_TRAIN_DEVICE_INDEX"] = str(lr)
            kw["device_id"] = torch.device("cuda", lr)
        backend = self.backend_config.backend or ("nccl" if use_gpu else "gloo")
        from .config import rccl_pg_options

        opts = rccl_pg_options(backend)
        if opts is not None:
            kw["pg_options"] = opts
        if world > 1:
            dist.init_process_group(backend, timeout=timedelta(seconds=self.backend_config.timeout_s), **kw)
